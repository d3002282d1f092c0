set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_generic_train_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_k10.log 2>&1 && \
timeout -k 10 300 python -u -m bench.fit_bench > gpurun_out/fit_bench.json 2> gpurun_out/fit_bench.err
echo EXIT $?
tail -4 gpurun_out/pytest_k10.log
cat gpurun_out/fit_bench.json
