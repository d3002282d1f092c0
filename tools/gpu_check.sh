#!/bin/bash
# One GPU call: selected GPU tests, then the headline bench (bench.py, 10 timed steps).
#   tools/gpu_check.sh tag "pytest selection"
set -o pipefail
tag=$1; sel=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $sel -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${tag}_tests.log | head -30
tail -2 gpurun_out/${tag}_tests.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo BENCH FAILED; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python tools/bench_brief.py gpurun_out/${tag}_bench.json
exit $rc
