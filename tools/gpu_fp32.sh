#!/bin/bash
# One GPU call: fp32-path GPU tests, then bench/fp32_micro.py (fp32 training / pooled inference timings).
#   tools/gpu_fp32.sh tag ["pytest selection"]
set -o pipefail
tag=$1; sel=${2:-tests/test_fp32_gpu.py}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $sel -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/${tag}_tests.log | grep -E "FAILED|ERROR" | head -30
tail -2 gpurun_out/${tag}_tests.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 400 python -m bench.fp32_micro > gpurun_out/${tag}_fp32micro.json 2> gpurun_out/${tag}_fp32micro.err \
  || { echo MICRO FAILED; tail -20 gpurun_out/${tag}_fp32micro.err; exit 1; }
cat gpurun_out/${tag}_fp32micro.json
exit $rc
