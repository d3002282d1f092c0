#!/bin/bash
# Probe-build A/B of the training step: training GPU tests on each probe .so, then bench/train_extra numbers
# for the library and each probe, interleaved over R rounds.
#   tools/probes/so_ab.sh tag rounds probe1 [probe2 ...]   (gpuprobe/<probe>.so)
set -o pipefail
tag=$1; rounds=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
for v in "$@"; do
  APNEAUQ_SO_PATH=$PWD/gpuprobe/$v.so timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_deterministic_gpu.py -m gpu -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_${v}_tests.log 2>&1
  rc=$?
  echo "== tests $v rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/${tag}_${v}_tests.log | head -10; tail -1 gpurun_out/${tag}_${v}_tests.log
  case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
done
for r in $(seq 1 $rounds); do
  for v in lib "$@"; do
    so=""; [ $v != lib ] && so=$PWD/gpuprobe/$v.so
    APNEAUQ_SO_PATH=$so timeout -k 10 300 python -c "
import json, torch
from bench import train_extra
o = train_extra.measure(torch.device('cuda'), 2025)
print('$v', json.dumps({k: o[k]['ms_per_step'] for k in ('single_b1024', 'single_b8192', 'members8_b1024')}), o['loss_parity']['max_rel'])
" 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
