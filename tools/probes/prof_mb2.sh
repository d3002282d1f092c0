# kernel-trace stats of the member-batched 8-member training step
cd /tmp && export TMPDIR=/tmp PYTHONPATH=/root/repo
R=/root/repo; OUT=$R/gpurun_out/prof_mb2; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/batched -o run -- python3 $R/bench/train_bench.py --members 8 --steps 20 --mode batched > $OUT/batched.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_mb2/batched/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
tot = sum(int(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms over 23 steps")
for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"]))[:30]:
    print(f"  {int(r['TotalDurationNs'])/1e6/23*1e3:8.1f} us/step  {int(r['Calls'])//23:3d}/step  {r['Name'][:80]}")
PY
