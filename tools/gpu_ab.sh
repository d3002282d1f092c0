#!/bin/bash
# One GPU call: per-kernel x3 times (rocprofv3) and interleaved x3_micro rounds of the library build vs
# probe builds.   tools/gpu_ab.sh tag probes_so/a.so ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 bash tools/probes/x3_abl.sh $tag default "$@" > gpurun_out/abl_$tag.txt 2>&1 || { echo ABL FAILED; tail -20 gpurun_out/abl_$tag.txt; exit 1; }
cat gpurun_out/abl_$tag.txt
timeout -k 10 600 bash tools/probes/x3_ab.sh 2 default "$@" -- --reps 3 2>&1 | grep -v amdgpu.ids
