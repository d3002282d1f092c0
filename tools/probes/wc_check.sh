set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/wc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wc_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/wc_tests.log | head -20; exit $rc; }
bash tools/probes/train_variants.sh wc
