#!/bin/bash
# Ping-pong forward phase ablations (probe builds in tools/probes/var2): 8 no conv, 16 no staging,
# 32 no epilogue/moments/copy-out, 48 = 16|32.
R=$(cd "$(dirname "$0")/../.." && pwd)
set -o pipefail
export PYTHONPATH=$R TMPDIR=/tmp
mkdir -p $R/gpurun_out
for v in main 8 16 32 48; do
  so=$R/tools/probes/var2/ppabl_$v.so; [ $v = main ] && so=$R/uncertaintyquantification_sleepapnea_1dcnn_amd/_apneauq_hip.so
  APNEAUQ_SO_PATH=$so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/gpurun_out/ppa_$v -o t -- python3 $R/tools/probes/fwd_abl.py $v > $R/gpurun_out/ppa_$v.json 2>/dev/null || exit 1
  echo "== $v $(cat $R/gpurun_out/ppa_$v.json)"
  f=$(find $R/gpurun_out/ppa_$v -name "*kernel_stats.csv" | head -1); python3 $R/tools/prof_summary.py $f 8 | grep fwd_
done
