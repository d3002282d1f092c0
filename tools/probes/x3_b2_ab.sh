# block 2 with 4 loader waves at 2-sample tiles (b2lw.so) vs the library's 4-sample tiles staged by MFMA waves
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
APNEAUQ_SO_PATH=/root/repo/probes_so/b2lw.so timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_b2.log 2>&1 && tail -2 gpurun_out/t_x3_b2.log || { tail -30 gpurun_out/t_x3_b2.log; exit 1; }
bash tools/probes/x3_abl.sh b2 default probes_so/b2lw.so > gpurun_out/abl_b2.txt 2>&1 && cat gpurun_out/abl_b2.txt
for r in 1 2; do
  echo -n "lib r$r: "; timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
  echo -n "b2lw r$r: "; APNEAUQ_SO_PATH=/root/repo/probes_so/b2lw.so timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
done
