#!/bin/bash
# One GPU call: kernel traces of the pooled-CNN fp32 inference modes (per-kernel totals over 2 reps).
set -o pipefail
tag=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in de mcd_batch mcd_running; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${tag}_fp$mode -o p -- \
    python3 /root/repo/bench/fp32_prof.py --mode $mode > /root/repo/gpurun_out/${tag}_fp$mode.log 2>&1 || { echo PROF FAILED; tail /root/repo/gpurun_out/${tag}_fp$mode.log; exit 1; }
  cd /root/repo
  f=$(find gpurun_out/${tag}_fp$mode -name "*kernel_stats.csv" | head -1)
  echo "== $mode"; python tools/prof_summary.py $f 14
done
