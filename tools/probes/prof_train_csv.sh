#!/bin/bash
# rocprofv3 kernel trace (csv) of bench.train_micro; busy/idle + per-kernel report.  $1 = tag
set -o pipefail
R=$PWD; export PYTHONPATH=$R
rm -rf $R/gpurun_out/ptc_$1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ptc_$1 -o t -- python3 -m bench.train_micro --steps 40 ${@:2} > $R/gpurun_out/ptc_$1.json 2> $R/gpurun_out/ptc_$1.err || exit 1
cd $R
tail -1 gpurun_out/ptc_$1.json
python3 tools/probes/gap_report.py $(find gpurun_out/ptc_$1 -name "*kernel_trace.csv" | head -1)
