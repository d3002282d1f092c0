set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m bench.generic_micro --n 16384 --T 50 > gpurun_out/generic_micro.json 2> gpurun_out/generic_micro.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gmicro -o gm -- python3 -m bench.generic_micro --n 16384 --T 10 --iters 2 > gpurun_out/prof_gmicro.log 2>&1
echo EXIT $?
cat gpurun_out/generic_micro.json
f=$(find gpurun_out/prof_gmicro -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 12
