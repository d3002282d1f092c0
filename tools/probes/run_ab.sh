# tests of the x3 engine, then per-kernel table + interleaved A/B of the library build vs probe builds
#   bash tools/probes/run_ab.sh <tag> <probe.so...>
set -o pipefail
cd /root/repo
tag=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_x3.log 2>&1 && tail -3 gpurun_out/t_x3.log &&
bash tools/probes/x3_abl.sh $tag default "$@" > gpurun_out/abl_$tag.txt 2>&1 && cat gpurun_out/abl_$tag.txt &&
bash tools/probes/x3_ab.sh 2 default "$@" -- --reps 3 2>&1 | grep -v amdgpu.ids
