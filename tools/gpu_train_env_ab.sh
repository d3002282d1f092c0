#!/bin/bash
# One GPU call: the training GPU tests, then bench/train_extra.py (the extra.train numbers) alternating
# between environment settings of the same build, R rounds.
#   tools/gpu_train_env_ab.sh tag rounds "VAR=a" "VAR=b" ...     ("-" = no extra variable)
set -o pipefail
tag=$1; rounds=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py -m gpu -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${tag}_tests.log | head -20
tail -2 gpurun_out/${tag}_tests.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
for r in $(seq 1 $rounds); do
  for e in "$@"; do
    if [ "$e" = "-" ]; then E=(); else E=("$e"); fi
    env "${E[@]}" timeout -k 10 300 python -c "
import json, torch
from bench import train_extra
o = train_extra.measure(torch.device('cuda'), 2025)
print('$e', json.dumps({k: o[k]['ms_per_step'] for k in ('single_b1024', 'single_b8192', 'members8_b1024')}), o['loss_parity']['max_rel'])
" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
exit $rc
