#!/bin/bash
# One GPU call: the whole GPU test tier (no -x: every failure of the run is reported), optionally
# restricted to a selection.   tools/gpu_suite.sh tag ["pytest selection"]
set -o pipefail
tag=$1; sel=${2:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest $sel -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/${tag}_tests.log | grep -E "FAILED|ERROR|SKIPPED" | head -40
tail -3 gpurun_out/${tag}_tests.log
exit $rc
