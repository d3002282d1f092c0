# training graph with wgrad on a forked stream (APNEAUQ_TRAIN_FORK=1) vs the serial chain
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
APNEAUQ_TRAIN_FORK=1 timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py -x -q --timeout 240 --timeout-method thread -k "graph or matches_autograd or reproducible" > gpurun_out/t_fork.log 2>&1; rc=$?; tail -3 gpurun_out/t_fork.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/t_fork.log | head; exit $rc; }
for r in 1 2 3; do
  echo -n "serial r$r: "; timeout -k 10 120 python3 bench/train_micro.py --batch 1024 --steps 50 || exit 1
  echo -n "fork r$r: "; APNEAUQ_TRAIN_FORK=1 timeout -k 10 120 python3 bench/train_micro.py --batch 1024 --steps 50 || exit 1
done
