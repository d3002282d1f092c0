# member-batched training (XCD-aware member placement, member-aware wgrad row groups): tests + A/B
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t_mb2.log 2>&1; rc=$?
tail -3 gpurun_out/t_mb2.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_mb2.log | head -20; exit $rc; }
for r in 1 2; do
  timeout -k 10 200 python3 bench/train_bench.py --members 8 --steps 30 --mode batched || exit 1
  timeout -k 10 200 python3 bench/train_bench.py --members 8 --steps 30 --mode streams || exit 1
done
timeout -k 10 200 python3 bench/train_bench.py --members 4 --steps 30 --mode batched || exit 1
timeout -k 10 200 python3 bench/train_bench.py --members 4 --steps 30 --mode streams || exit 1
