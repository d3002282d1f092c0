# fused pooled kernel: library build vs a probe .so ($1), tests + 2 interleaved micro-bench rounds
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo
timeout -k 10 300 python -u -m pytest tests/test_fused_tiled_gpu.py tests/test_generic_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pooled.log 2>&1 && tail -2 gpurun_out/t_pooled.log || { tail -40 gpurun_out/t_pooled.log; exit 1; }
for r in 1 2; do
  echo "lib r$r: $(timeout -k 10 200 python3 bench/generic_micro.py --iters 5 2>/dev/null | tr -d '\n ')" || exit 1
  echo "probe r$r: $(APNEAUQ_SO_PATH=/root/repo/$1 timeout -k 10 200 python3 bench/generic_micro.py --iters 5 2>/dev/null | tr -d '\n ')" || exit 1
done
