# fused pooled-CNN kernel: GPU tests, micro-bench against the layer-wise path, kernel trace
set -o pipefail
cd /root/repo
export PYTHONPATH=/root/repo TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_tiled_gpu.py tests/test_generic_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_pooled.log 2>&1 && tail -3 gpurun_out/t_pooled.log || { tail -40 gpurun_out/t_pooled.log; exit 1; }
timeout -k 10 300 python3 bench/generic_micro.py > gpurun_out/generic_micro_pooled.json 2>gpurun_out/generic_micro_pooled.err && cat gpurun_out/generic_micro_pooled.json || { tail -20 gpurun_out/generic_micro_pooled.err; exit 1; }
rm -rf gpurun_out/prof_pooled
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pooled -o run -- python3 bench/generic_micro.py --iters 1 > gpurun_out/prof_pooled.log 2>&1 && echo prof-ok
