set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bnbatch -o bb -- python3 bench.py --bn-mode batch --steps 3 --warmup 1 > gpurun_out/prof_bnbatch.log 2>&1
echo EXIT $?
f=$(find gpurun_out/prof_bnbatch -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 14
