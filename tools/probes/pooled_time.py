"""Kernel time of the fused pooled CNN (csrc/fused_tiled.hip) for MC Dropout T=50 x 16384 windows,
dropout on / off (APNEAUQ_SO_PATH selects a probe build)."""
import dataclasses
import json
import sys

import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, fused

spec = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                      for i, b in enumerate(DEFAULT_SPEC.blocks)))
p = {k: v.cuda() for k, v in R.synthetic_params(spec, 1).items()}
blob = fused.pack_blob(spec, p).unsqueeze(0)
x = torch.randn(16384, 60, 4, device="cuda").to(torch.bfloat16)
thr, dsc = fused.dropout_tables(spec)
o = _ext.ops()
res = {}
for drop in (True, False):
    f = lambda: o.fused_pooled_forward(x, blob, 50, 0, 0, 3, drop, False, thr, dsc)  # noqa: E731
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        f()
    e1.record()
    torch.cuda.synchronize()
    res["drop" if drop else "nodrop"] = round(e0.elapsed_time(e1) / 5, 3)
print(json.dumps({"so": sys.argv[1] if len(sys.argv) > 1 else "lib", **res}))
