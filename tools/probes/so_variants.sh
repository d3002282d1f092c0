#!/bin/bash
# Kernel stats (rocprofv3) of bench.train_micro for every probe build tools/probes/sovar/<prefix>*.so
#   $1 = prefix, $2 = batch, $3 = kernel-name grep pattern
set -e
R=$PWD; export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for so in $R/tools/probes/sovar/$1*.so; do
  tag=$(basename $so .so)
  rm -rf $R/gpurun_out/sv_$tag
  APNEAUQ_SO_PATH=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/sv_$tag -o t -- python3 -m bench.train_micro --steps 5 --batch $2 > $R/gpurun_out/sv_$tag.json 2>/dev/null
  echo "== $tag $(cat $R/gpurun_out/sv_$tag.json)"
  python3 $R/tools/probes/db_top.py $R/gpurun_out/sv_$tag 40 | grep -E "$3" || true
done
