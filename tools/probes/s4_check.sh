# full GPU check of the tree: smoke, GPU suite, headline bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/s4_smoke.log; exit 1; }
tail -1 gpurun_out/s4_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/s4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s4_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/s4_tests.log | head; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/s4_bench.json 2> gpurun_out/s4_bench.err && cat gpurun_out/s4_bench.json
