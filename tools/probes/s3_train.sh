set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py tests/test_rccl_gpu.py tests/test_distributed_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/s3t_tests.log 2>&1
rc=$?; tail -4 gpurun_out/s3t_tests.log
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|error|assert|FAILED" gpurun_out/s3t_tests.log | head -30; exit $rc; }
timeout -k 10 200 python -m bench.train_micro --steps 50 | tail -1 && bash tools/probes/prof_train_csv.sh b | head -12
