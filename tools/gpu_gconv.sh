set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_generic_gpu.py tests/test_generic_train_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gconv.log 2>&1 && \
timeout -k 10 300 python -u -m bench.generic_micro --n 16384 --T 50 > gpurun_out/generic_micro.json 2> gpurun_out/generic_micro.err && \
timeout -k 10 300 python -u -m bench.generic_train_micro --no-torch > gpurun_out/gtrain_micro.json 2> gpurun_out/gtrain_micro.err
echo EXIT $?
tail -4 gpurun_out/pytest_gconv.log
cat gpurun_out/generic_micro.json gpurun_out/gtrain_micro.json
