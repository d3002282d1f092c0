#!/bin/bash
# wgrad kernel times of probe builds (kernel trace of bench.train_micro): tools/probes/wg_var.sh <batch> so...
set -o pipefail
R=/root/repo; export PYTHONPATH=$R TMPDIR=/tmp; b=$1; shift
for so in main "$@"; do
  if [ $so = main ]; then unset APNEAUQ_SO_PATH; else export APNEAUQ_SO_PATH=$R/$so; fi
  n=$(basename $so .so)_$b; rm -rf $R/gpurun_out/wv_$n
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/wv_$n -o t -- python3 -m bench.train_micro --steps 30 --batch $b > $R/gpurun_out/wv_$n.json 2> $R/gpurun_out/wv_$n.err) || exit 1
  echo "== $n $(tail -1 $R/gpurun_out/wv_$n.json | cut -c1-90)"
  python3 $R/tools/probes/gap_report.py $(find $R/gpurun_out/wv_$n -name "*kernel_trace.csv" | head -1) | grep -E "span|wgrad_kernel|dgrad_kernel<4" | cut -c1-100
done
