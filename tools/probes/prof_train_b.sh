#!/bin/bash
# rocprofv3 kernel stats of bench.train_micro at batch $2; $1 = output tag.
set -e
R=$PWD; export PYTHONPATH=$R
rm -rf $R/gpurun_out/prof_$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$1 -o train -- python3 -m bench.train_micro --steps 10 --batch $2 > $R/gpurun_out/train_micro_$1.json 2> $R/gpurun_out/train_prof_$1.err
cd $R
cat gpurun_out/train_micro_$1.json
python3 tools/probes/db_top.py gpurun_out/prof_$1 20
