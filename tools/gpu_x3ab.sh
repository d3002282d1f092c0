#!/bin/bash
# One GPU call: x3 GPU tests on the library build, then per-kernel x3 times (rocprofv3) of the library
# build vs probe builds.   tools/gpu_x3ab.sh tag gpuprobe/a.so ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_x3_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_x3tests.log 2>&1 || { echo X3 TESTS FAILED; tail -30 gpurun_out/${tag}_x3tests.log; exit 1; }
tail -2 gpurun_out/${tag}_x3tests.log
timeout -k 10 500 bash tools/probes/x3_abl.sh $tag default "$@" > gpurun_out/abl_$tag.txt 2>&1 || { echo ABL FAILED; tail -20 gpurun_out/abl_$tag.txt; exit 1; }
cat gpurun_out/abl_$tag.txt
