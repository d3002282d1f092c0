#!/bin/bash
# L1 / texture-path counters of the layer-wise forward kernels (ping-pong vs single-team).
R=$(cd "$(dirname "$0")/../.." && pwd)
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for pp in 1 0; do
  OUT=$R/gpurun_out/pmc_tcp_$pp; rm -rf $OUT; mkdir -p $OUT
  APNEAUQ_FWD_PP=$pp timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT -o run -- python3 $R/tools/probes/fwd_abl.py pp$pp > $OUT.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for pp in (1, 0):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/pmc_tcp_{pp}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "fwd" in k:
                agg[k[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    print("== pp", pp)
    for k, v in sorted(agg.items()):
        print(k, {n: f"{x:.3g}" for n, x in sorted(v.items())})
PY
