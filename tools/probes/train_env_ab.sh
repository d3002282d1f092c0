#!/bin/bash
# Interleaved bench.train_micro rounds (batch 8192 and 1024) under environment arms:
#   tools/probes/train_env_ab.sh <rounds> default VAR=VAL ...
set -o pipefail
n=$1; shift
export PYTHONPATH=$PWD
for rep in $(seq 1 $n); do
  for arm in "$@"; do
    if [ "$arm" = default ]; then e=(); else e=("$arm"); fi
    a=$(env "${e[@]}" timeout -k 10 200 python3 -m bench.train_micro --batch 8192 --steps 30 2>/dev/null | tail -1) || exit 1
    b=$(env "${e[@]}" timeout -k 10 200 python3 -m bench.train_micro --batch 1024 --steps 100 2>/dev/null | tail -1) || exit 1
    echo "$rep $arm b8192 $(echo $a | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"], 4))') ms | b1024 $(echo $b | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_per_step"], 4))') ms"
  done
done
