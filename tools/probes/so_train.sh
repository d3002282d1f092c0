#!/bin/bash
# Training-step time (bench.train_micro, HIP graph) and the batch-BN chunk for the library build and
# every probe build tools/probes/sovar/<prefix>*.so:   tools/probes/so_train.sh <prefix>
set -o pipefail
R=$PWD; export PYTHONPATH=$R TMPDIR=/tmp
for so in $R/uncertaintyquantification_sleepapnea_1dcnn_amd/_apneauq_hip.so $R/tools/probes/sovar/$1*.so; do
  tag=$(basename $so .so)
  echo "== $tag $(APNEAUQ_SO_PATH=$so timeout -k 10 120 python3 -m bench.train_micro --steps 100) $(APNEAUQ_SO_PATH=$so timeout -k 10 120 python3 tools/probes/fwd_abl.py $tag)" || exit 1
done
