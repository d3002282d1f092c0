# pair-split forward variants: correctness of the all-layers variant, then the headline bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
APNEAUQ_SO_PATH=$PWD/tools/probes/sovar/half44.so timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q \
  -k "batch_stats or autograd or moments or pingpong or reduces" --timeout 240 --timeout-method thread > gpurun_out/half_tests.log 2>&1
rc=$?; tail -3 gpurun_out/half_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/half_tests.log | head -20; exit $rc; }
bash tools/probes/so_bench1.sh half 2
