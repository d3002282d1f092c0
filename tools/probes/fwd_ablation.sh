#!/bin/bash
# Build probe variants of the layer-wise forward kernels (CPU side) -- run with "build" here, then on
# the GPU box without arguments: times one 16-pass batch-BN MC-Dropout chunk per variant + kernel stats.
R=$(cd "$(dirname "$0")/../.." && pwd)
VARS=${VARS:-"0 4 8 16 32 20 12"}
if [ "$1" = build ]; then
  mkdir -p $R/tools/probes/sovar
  for v in $VARS; do
    APNEAUQ_SO_OUT=$R/tools/probes/sovar/fwdabl_$v.so APNEAUQ_HIPCC_FLAGS="-DAPNEAUQ_FWD_ABL=$v" \
      python -m uncertaintyquantification_sleepapnea_1dcnn_amd.csrc.build > /dev/null || exit 1
  done
  exit 0
fi
set -o pipefail
export PYTHONPATH=$R TMPDIR=/tmp
mkdir -p $R/gpurun_out
for v in $VARS; do
  APNEAUQ_SO_PATH=$R/tools/probes/sovar/fwdabl_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/gpurun_out/fa_$v -o t -- python3 $R/tools/probes/fwd_abl.py $v > $R/gpurun_out/fa_$v.json 2>$R/gpurun_out/fa_$v.err || exit 1
  echo "== ABL $v $(cat $R/gpurun_out/fa_$v.json)"
  f=$(find $R/gpurun_out/fa_$v -name "*kernel_stats.csv" | head -1); python3 $R/tools/prof_summary.py $f 8 | grep fwd_kernel
done
