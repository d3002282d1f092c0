#!/bin/bash
# Ping-pong forward: batch-stats tests, one 16-pass chunk under rocprofv3 kernel stats, the bench.
R=$(cd "$(dirname "$0")/../.." && pwd)
set -o pipefail
export PYTHONPATH=$R TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "batch_stats or moments or matches_autograd or pingpong" > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -2 gpurun_out/pp_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp_prof -o t -- python3 $R/tools/probes/fwd_abl.py pp > $R/gpurun_out/pp.json 2>/dev/null || exit 1
echo "== $(cat $R/gpurun_out/pp.json)"
f=$(find $R/gpurun_out/pp_prof -name "*kernel_stats.csv" | head -1); python3 $R/tools/prof_summary.py $f 10
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 > gpurun_out/pp_bench.json 2> gpurun_out/pp_bench.err || { tail -20 gpurun_out/pp_bench.err; exit 1; }
cat gpurun_out/pp_bench.json
