set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_generic_train_gpu.py tests/test_generic_gpu.py tests/test_train_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gtrain.log 2>&1
echo EXIT $?
tail -30 gpurun_out/pytest_gtrain.log
