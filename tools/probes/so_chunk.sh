#!/bin/bash
# Batch-BN chunk timing + per-kernel stats for the library build and every probe build
# tools/probes/sovar/<prefix>*.so:   tools/probes/so_chunk.sh <prefix>
set -o pipefail
R=$PWD; export PYTHONPATH=$R TMPDIR=/tmp
mkdir -p gpurun_out
for so in $R/uncertaintyquantification_sleepapnea_1dcnn_amd/_apneauq_hip.so $R/tools/probes/sovar/$1*.so; do
  tag=$(basename $so .so)
  APNEAUQ_SO_PATH=$so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sc_$tag -o t -- python3 $R/tools/probes/fwd_abl.py $tag > $R/gpurun_out/sc_$tag.json 2> $R/gpurun_out/sc_$tag.err || { echo "FAIL $tag"; tail -5 $R/gpurun_out/sc_$tag.err; exit 1; }
  echo "== $(cat $R/gpurun_out/sc_$tag.json)"
  f=$(find $R/gpurun_out/sc_$tag -name "*kernel_stats.csv" | head -1); python3 $R/tools/prof_summary.py $f 8 | grep -E "fwd_kernel<[1-5]>" | awk -F'|' '{printf "%s %s\n", $2, $5}'
done
