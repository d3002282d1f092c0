#!/bin/bash
# One GPU call: the GPU test tier, the headline bench and a kernel-trace profile of it.
#   tools/gpu_check.sh [tag] [pytest selection...]
set -o pipefail
tag=${1:-chk}; shift
sel=${@:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|error|assert" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o p -- python3 bench.py --steps 3 --warmup 1 --no-deviation > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF FAILED; tail gpurun_out/${tag}_prof.log; exit 1; }
f=$(find gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 16
