#!/bin/bash
# One GPU call: selected GPU tests, then the x3 A/B (tools/gpu_ab.sh) of probe builds.
#   tools/gpu_tests_ab.sh tag "pytest selection" so1 so2 ...
set -o pipefail
tag=$1; sel=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $sel -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${tag}_tests.log | head -30
tail -2 gpurun_out/${tag}_tests.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
bash tools/gpu_ab.sh $tag "$@" || exit $?
exit $rc
