#!/bin/bash
# One GPU call: selected GPU tests, then the headline bench (and optionally a kernel-trace profile).
#   tools/gpu_quick.sh tag "pytest selection" [prof]
set -o pipefail
tag=$1; sel=$2; prof=$3
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; grep -E "Error|error|assert|FAILED" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));e=d['extra'];print('value',d['value'],'mcd',e['mcd_phase_ms'],'de',e['de_phase_ms'],'running',e['running_bn']['value'],e['running_bn']['mcd_phase_ms']);print('dev',json.dumps(e['fp32_deviation']['mcd_batch_bn']['max_abs_dp']),json.dumps(e['fp32_deviation']['mcd_batch_bn']['aggregates_delta']))"
if [ -n "$prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o p -- python3 bench.py --steps 3 --warmup 1 --no-deviation > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF FAILED; tail gpurun_out/${tag}_prof.log; exit 1; }
  f=$(find gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 14
fi
