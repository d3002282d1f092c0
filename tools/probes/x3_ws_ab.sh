# x3 batch-BN MCD vs activation-workspace cap (pass chunking) + numerics of the key hoisting
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_uq_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3_ws.log 2>&1 && tail -2 gpurun_out/t_x3_ws.log || { tail -30 gpurun_out/t_x3_ws.log; exit 1; }
for r in 1 2; do
  for gb in 100 24 12; do
    echo -n "ws ${gb} GB r$r: "; APNEAUQ_X3_WS_GB=$gb timeout -k 10 200 python3 bench/x3_micro.py --reps 3 --only mcd || exit 1
  done
done
