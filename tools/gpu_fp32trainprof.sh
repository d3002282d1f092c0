set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for mode in train mcd_batch; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/fpt_$mode -o p -- \
    python3 /root/repo/bench/fp32_prof.py --mode $mode > /root/repo/gpurun_out/fpt_$mode.log 2>&1 || { echo PROF FAILED; tail /root/repo/gpurun_out/fpt_$mode.log; exit 1; }
  cd /root/repo
  f=$(find gpurun_out/fpt_$mode -name "*kernel_stats.csv" | head -1)
  echo "== $mode"; python tools/prof_summary.py $f 22
done
