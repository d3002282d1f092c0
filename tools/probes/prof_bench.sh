#!/bin/bash
# rocprofv3 kernel stats of bench.py; $1 = output tag, remaining args go to bench.py.
set -e
tag=$1; shift
R=$PWD; export PYTHONPATH=$R
rm -rf $R/gpurun_out/prof_$tag
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o bench -- python3 $R/bench.py "$@" > $R/gpurun_out/bench_$tag.json 2> $R/gpurun_out/bench_prof_$tag.err
cd $R
cat gpurun_out/bench_$tag.json
python3 tools/probes/db_top.py gpurun_out/prof_$tag 16
