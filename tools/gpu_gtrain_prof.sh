set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in pooled single30; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gtrain_$s -o gt -- python3 -m bench.generic_train_micro --specs $s --iters 10 --no-torch > gpurun_out/prof_gtrain_$s.log 2>&1 || exit 1
f=$(find gpurun_out/prof_gtrain_$s -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f 25 > gpurun_out/gtrain_kstats_$s.md
done
echo EXIT $?
cat gpurun_out/gtrain_kstats_*.md
