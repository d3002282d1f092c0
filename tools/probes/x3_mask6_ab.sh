# block 5's output mask drawn by block 6's loader waves (APNEAUQ_X3_MASK6=1) vs block 5's epilogue
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
APNEAUQ_X3_MASK6=1 timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_m6.log 2>&1 && tail -2 gpurun_out/t_m6.log || { tail -30 gpurun_out/t_m6.log; exit 1; }
for r in 1 2 3; do
  echo -n "epi r$r: "; timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
  echo -n "mask6 r$r: "; APNEAUQ_X3_MASK6=1 timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
done
