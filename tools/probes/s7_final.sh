# final check of the tree: smoke, GPU suite, bench with the driver's arguments, training benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=/root/repo
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s6_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/s6_smoke.log; exit 1; }
tail -1 gpurun_out/s6_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/s6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s6_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/s6_tests.log | head; exit $rc; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s6_bench.json 2> gpurun_out/s6_bench.err && cat gpurun_out/s6_bench.json &&
timeout -k 10 200 python3 bench/train_bench.py --members 8 --steps 30 --mode batched &&
timeout -k 10 200 python3 bench/train_micro.py --batch 1024 --steps 50
