set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_generic_train_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gtrain.log 2>&1 && \
timeout -k 10 300 python -u -m bench.generic_train_micro > gpurun_out/gtrain_micro.json 2> gpurun_out/gtrain_micro.err
echo EXIT $?
tail -5 gpurun_out/pytest_gtrain.log
cat gpurun_out/gtrain_micro.json
