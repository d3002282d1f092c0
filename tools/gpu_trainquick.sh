#!/bin/bash
# One GPU call: the training GPU tests, then bench/train_extra.py measured twice (extra.train numbers).
#   tools/gpu_trainquick.sh tag
set -o pipefail
tag=$1
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py -m gpu -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${tag}_tests.log | head -20
tail -2 gpurun_out/${tag}_tests.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
for r in 1 2; do
  timeout -k 10 300 python -c "
import json, torch
from bench import train_extra
o = train_extra.measure(torch.device('cuda'), 2025)
print(json.dumps({k: o[k] for k in ('single_b1024', 'single_b8192', 'members8_b1024')}))
print(json.dumps(o['loss_parity']['max_rel']))
" || exit 1
done
exit $rc
