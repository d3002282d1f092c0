#!/bin/bash
# generic training step vs the wgrad's minimum chunks per workgroup (APNEAUQ_GWG_MINC; 0 = default)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
for v in 4 0 8 16 32; do
  echo "== minc=$v"; APNEAUQ_GWG_MINC=$v timeout -k 10 200 python3 -m bench.generic_train_micro --specs pooled,single30 --iters 50 --no-torch | grep -E '"(pooled|single30)"|hip_generic_ms"' || exit 1
done
