#!/bin/bash
# One GPU iteration: batch-BN chunk timing (library build) + kernel stats, then the selected GPU tests
# and the headline bench.   tools/gpu_iter.sh <tag> [pytest selection]
set -o pipefail
tag=${1:-it}; shift
sel=${@:-tests}
R=$PWD; export PYTHONPATH=$R TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_fa -o t -- python3 tools/probes/fwd_abl.py $tag > gpurun_out/${tag}_fa.json 2> gpurun_out/${tag}_fa.err || { echo FA FAILED; tail gpurun_out/${tag}_fa.err; exit 1; }
cat gpurun_out/${tag}_fa.json
f=$(find gpurun_out/${tag}_fa -name "*kernel_stats.csv" | head -1); python3 tools/prof_summary.py $f 10
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|error|assert|FAIL" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-deviation > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));e=d['extra'];print('value',d['value'],'mcd',e['mcd_phase_ms'],'de',e['de_phase_ms'],'running',e['running_bn']['value'])"
