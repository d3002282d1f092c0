# kernel-trace stats: member-batched 8-member step vs one model at batch 8192 vs streams
cd /tmp && export TMPDIR=/tmp PYTHONPATH=/root/repo
R=/root/repo; OUT=$R/gpurun_out/prof_mb; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/batched -o run -- python3 $R/bench/train_bench.py --members 8 --steps 20 --mode batched > $OUT/batched.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b8192 -o run -- python3 $R/bench/train_micro.py --batch 8192 --steps 20 > $OUT/b8192.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/streams -o run -- python3 $R/bench/train_bench.py --members 8 --steps 20 --mode streams > $OUT/streams.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob, os
for tag in ("batched", "b8192", "streams"):
    f = glob.glob(f"gpurun_out/prof_mb/{tag}/**/*kernel_stats.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    tot = sum(int(r["TotalDurationNs"]) for r in rows)
    print(f"== {tag}: total kernel time {tot/1e6:.2f} ms")
    for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"]))[:22]:
        print(f"  {int(r['TotalDurationNs'])/1e6:8.2f} ms  {int(r['Calls']):6d} calls  {r['Name'][:90]}")
PY
