set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --bn-mode batch > gpurun_out/bench_batch.log 2>&1
echo EXIT $?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log | tail -2; tail -1 gpurun_out/bench.log; tail -1 gpurun_out/bench_batch.log
