#!/bin/bash
# bench/train_extra.measure (single b1024 / b8192, 8 members) for the library build and probe builds,
# interleaved: tools/probes/train_extra_ab.sh <rounds> so...
set -o pipefail
n=$1; shift
export PYTHONPATH=$PWD
for rep in $(seq 1 $n); do
  for so in main "$@"; do
    if [ $so = main ]; then unset APNEAUQ_SO_PATH; else export APNEAUQ_SO_PATH=$PWD/$so; fi
    r=$(timeout -k 10 300 python3 -c "
import json, torch
from bench import train_extra
d = train_extra.measure(torch.device('cuda'), steps=30)
print(json.dumps({k: v['ms_per_step'] for k, v in d.items() if isinstance(v, dict) and 'ms_per_step' in v}))
" 2>/dev/null | tail -1) || exit 1
    echo "$rep $(basename $so .so) $r"
  done
done
