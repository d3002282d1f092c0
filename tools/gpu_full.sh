#!/bin/bash
# One GPU call: the WHOLE GPU test tier, then bench.py (driver defaults) and a kernel-trace profile of it.
#   tools/gpu_full.sh tag
set -o pipefail
tag=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${tag}_suite.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${tag}_suite.log | head -30
tail -2 gpurun_out/${tag}_suite.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo BENCH FAILED; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python tools/bench_brief.py gpurun_out/${tag}_bench.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${tag}_prof -o p -- \
  python3 /root/repo/bench.py --steps 3 --warmup 1 --no-deviation > /root/repo/gpurun_out/${tag}_prof.log 2>&1 \
  || { echo PROF FAILED; tail /root/repo/gpurun_out/${tag}_prof.log; exit 1; }
cd /root/repo
f=$(find gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 30
exit $rc
