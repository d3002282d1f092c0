# 64-channel chunks: library (block 3 at CK 64) vs ck32.so (all 32) vs ck6.so (blocks 3 and 6 at 64)
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_ck.log 2>&1 && tail -2 gpurun_out/t_x3_ck.log || { tail -30 gpurun_out/t_x3_ck.log; exit 1; }
APNEAUQ_SO_PATH=/root/repo/probes_so/ck6.so timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_ck6.log 2>&1 && tail -2 gpurun_out/t_x3_ck6.log || { tail -30 gpurun_out/t_x3_ck6.log; exit 1; }
bash tools/probes/x3_abl.sh ck default probes_so/ck32.so probes_so/ck6.so > gpurun_out/abl_ck.txt 2>&1 && cat gpurun_out/abl_ck.txt
for r in 1 2; do
  echo -n "lib r$r: "; timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de || exit 1
  echo -n "ck32 r$r: "; APNEAUQ_SO_PATH=/root/repo/probes_so/ck32.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de || exit 1
  echo -n "ck6 r$r: "; APNEAUQ_SO_PATH=/root/repo/probes_so/ck6.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd,de || exit 1
done
