#!/bin/bash
# One GPU call: kernel traces of the training step at batch 1024 and 8192 (per-kernel us per step).
#   tools/gpu_trainprof.sh tag [--fp32]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 1024 8192; do
  s=$([ $b = 1024 ] && echo 40 || echo 12)
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${tag}_tp$b -o p -- \
    python3 /root/repo/bench/train_prof.py --batch $b --steps $s "$@" > /root/repo/gpurun_out/${tag}_tp$b.log 2>&1 || { echo PROF FAILED; tail /root/repo/gpurun_out/${tag}_tp$b.log; exit 1; }
  cd /root/repo
  f=$(find gpurun_out/${tag}_tp$b -name "*kernel_stats.csv" | head -1)
  echo "== batch $b ($s steps)"; python tools/prof_summary.py $f 28
done
