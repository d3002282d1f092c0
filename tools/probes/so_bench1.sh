#!/bin/bash
# Headline bench (--no-secondary --no-deviation) for the in-tree .so and each tools/probes/sovar/<prefix>*.so,
# interleaved over $2 rounds
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${2:-2}); do
  for so in main tools/probes/sovar/$1*.so; do
    tag=$(basename $so .so)
    if [ $so = main ]; then unset APNEAUQ_SO_PATH; else export APNEAUQ_SO_PATH=$PWD/$so; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-secondary --no-deviation > gpurun_out/sb1_$tag.json 2>gpurun_out/sb1_$tag.err || { echo "FAIL $tag"; tail -5 gpurun_out/sb1_$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/sb1_$tag.json'));print('$rep $tag', d['value'], d['extra']['mcd_phase_ms'], d['extra']['de_phase_ms'])"
  done
done
