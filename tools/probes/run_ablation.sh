#!/bin/bash
# Run every built ablation variant of the fused kernel (tools/probes/bin/abl_*), MCD then DE,
# ${REPS:-1} interleaved rounds (A/B comparisons must come from the same box and call).
set -e
mkdir -p gpurun_out
out=gpurun_out/ablation.jsonl
: > $out
for rep in $(seq ${REPS:-1}); do
  for b in tools/probes/bin/abl_*; do
    echo -n "{\"bin\": \"$(basename $b)\", \"r\": " >> $out
    timeout -k 10 60 $b mcd >> $out
    echo -n "{\"bin\": \"$(basename $b)\", \"r\": " >> $out
    timeout -k 10 60 $b de >> $out
  done
done
cat $out
