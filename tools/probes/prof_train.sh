#!/bin/bash
# rocprofv3 kernel stats of bench.train_micro; $1 = output tag, $2 = batch (1024), $3 = precision (bf16).  Prints the top kernels.
set -e
R=$PWD; export PYTHONPATH=$R
rm -rf $R/gpurun_out/prof_$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$1 -o train -- python3 -m bench.train_micro --steps 20 --batch ${2:-1024} --precision ${3:-bf16} > $R/gpurun_out/train_micro_$1.json 2> $R/gpurun_out/train_prof_$1.err
cd $R
cat gpurun_out/train_micro_$1.json
python3 tools/probes/db_top.py gpurun_out/prof_$1 14
