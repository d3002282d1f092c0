# x3 engine check on the GPU box: numerics tests, headline bench, per-kernel table + counters
set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py tests/test_prep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3.log 2>&1 && tail -2 gpurun_out/t_x3.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_x3.json 2> gpurun_out/bench_x3.err && cat gpurun_out/bench_x3.json &&
bash tools/probes/x3_abl.sh final default > gpurun_out/abl_final.txt 2>&1 && cat gpurun_out/abl_final.txt &&
bash tools/probes/x3_pmc_tcp.sh > gpurun_out/pmc_final.txt 2>&1 && cat gpurun_out/pmc_final.txt
