set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
for r in 1 2; do
for g in 4 2 1 8; do
timeout -k 10 300 python -c "
import json, torch
from bench import train_extra
o = train_extra.measure(torch.device('cuda'), 2025, groups=$g)
print($g, o['members8_b1024']['ms_per_step'])
" 2>&1 | grep -v amdgpu.ids || exit 1
done; done
