#!/bin/bash
# One GPU call: training GPU tests, then kernel traces of the training step at batch 1024 and 8192 under
# each environment setting (per-kernel us; SKIP_TESTS=1 skips the tests).
#   tools/gpu_trainprof_env.sh tag "-" "VAR=value" ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=/root/repo
rc=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py -m gpu -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" gpurun_out/${tag}_tests.log | head -20
  tail -1 gpurun_out/${tag}_tests.log
fi
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
i=0
for e in "$@"; do
  i=$((i+1))
  for b in 1024 8192; do
    s=$([ $b = 1024 ] && echo 40 || echo 12)
    if [ "$e" = "-" ]; then unset APNEAUQ_TRAIN_FWD APNEAUQ_TRAIN_FUSED_REDUCE; else export "$e"; fi
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${tag}_e${i}_$b -o p -- \
      python3 /root/repo/bench/train_prof.py --batch $b --steps $s > /root/repo/gpurun_out/${tag}_e${i}_$b.log 2>&1 || { echo PROF FAILED; exit 1; }
    cd /root/repo
    f=$(find gpurun_out/${tag}_e${i}_$b -name "*kernel_stats.csv" | head -1)
    echo "== $e batch $b ($s steps)"
    python3 - "$f" "$s" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
tot = 0.0
for r in rows:
    n = r["Name"]
    us = float(r["TotalDurationNs"]) / 1e3 / steps
    tot += us
    if us >= 1.0:
        print(f"  {us:8.1f} us/step  {n[:70]}")
print(f"  total kernel time {tot:.1f} us/step")
PY
  done
done
unset APNEAUQ_TRAIN_FWD APNEAUQ_TRAIN_FUSED_REDUCE
exit $rc
