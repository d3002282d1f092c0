#!/bin/bash
# Kernel trace (csv) of bench.train_micro from another checkout: $1 = tag, $2 = tree ("." = this one),
# the rest = train_micro args.  Prints the gap report (busy / per-kernel times).
set -o pipefail
R=/root/repo; T=$R/$2; tag=$1; shift 2
rm -rf $R/gpurun_out/pt_$tag
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$T timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pt_$tag -o t -- python3 -m bench.train_micro --steps 40 "$@" > $R/gpurun_out/pt_$tag.json 2> $R/gpurun_out/pt_$tag.err || exit 1
cd $R
tail -1 gpurun_out/pt_$tag.json
python3 tools/probes/gap_report.py $(find gpurun_out/pt_$tag -name "*kernel_trace.csv" | head -1)
