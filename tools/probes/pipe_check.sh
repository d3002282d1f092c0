#!/bin/bash
# Forward-kernel staging variants: tests on the main build, then one 16-pass batch-BN chunk per
# variant (.so via APNEAUQ_SO_PATH) under rocprofv3 kernel stats.
R=$(cd "$(dirname "$0")/../.." && pwd)
set -o pipefail
export PYTHONPATH=$R TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "batch_stats or moments or matches_autograd" > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -2 gpurun_out/pipe_tests.log
for v in main prio delay pipe1; do
  so=$R/tools/probes/var2/$v.so; [ $v = main ] && so=$R/uncertaintyquantification_sleepapnea_1dcnn_amd/_apneauq_hip.so
  APNEAUQ_SO_PATH=$so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/gpurun_out/pv_$v -o t -- python3 $R/tools/probes/fwd_abl.py $v > $R/gpurun_out/pv_$v.json 2>/dev/null || exit 1
  echo "== $v $(cat $R/gpurun_out/pv_$v.json)"
  f=$(find $R/gpurun_out/pv_$v -name "*kernel_stats.csv" | head -1); python3 $R/tools/prof_summary.py $f 8 | grep fwd_kernel
done
