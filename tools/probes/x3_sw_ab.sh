# block 2 (no loader waves): staging spread over all 8 MFMA waves (sw8.so) vs waves 0-3 (library)
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
APNEAUQ_SO_PATH=/root/repo/probes_so/sw8.so timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_sw.log 2>&1 && tail -2 gpurun_out/t_x3_sw.log || { tail -30 gpurun_out/t_x3_sw.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_lib.log 2>&1 && tail -2 gpurun_out/t_x3_lib.log || { tail -30 gpurun_out/t_x3_lib.log; exit 1; }
bash tools/probes/x3_abl.sh sw default probes_so/sw8.so > gpurun_out/abl_sw.txt 2>&1 && cat gpurun_out/abl_sw.txt
for r in 1 2; do
  echo -n "lib r$r: "; timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
  echo -n "sw8 r$r: "; APNEAUQ_SO_PATH=/root/repo/probes_so/sw8.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
done
