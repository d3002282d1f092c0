# A/B of the generic inference conv: LDS-staged kernel (default) vs the direct-gather kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_generic_gpu.py tests/test_generic_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gconv.log 2>&1 && \
timeout -k 10 300 python -u -m bench.generic_micro --n 16384 --T 50 > gpurun_out/generic_micro_lds.json 2> gpurun_out/generic_micro.err && \
APNEAUQ_GCONV_LDS=0 timeout -k 10 300 python -u -m bench.generic_micro --n 16384 --T 50 > gpurun_out/generic_micro_gather.json 2>> gpurun_out/generic_micro.err && \
timeout -k 10 300 python -u -m bench.generic_train_micro --no-torch > gpurun_out/gtrain_micro.json 2> gpurun_out/gtrain_micro.err
echo EXIT $?
tail -3 gpurun_out/pytest_gconv.log
cat gpurun_out/generic_micro_lds.json gpurun_out/generic_micro_gather.json gpurun_out/gtrain_micro.json
