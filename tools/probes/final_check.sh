set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/fc_smoke.log; exit 1; }
tail -1 gpurun_out/fc_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/fc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fc_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/fc_tests.log | head; exit $rc; }
