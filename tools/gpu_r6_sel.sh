set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_fp32_gpu.py tests/test_x3_gpu.py tests/test_generic_train_gpu.py tests/test_train_gpu.py tests/test_deterministic_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6b_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/r6b_tests.log | head -20
tail -2 gpurun_out/r6b_tests.log
exit $rc
