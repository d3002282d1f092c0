"""Fused x3 kernel: does a loud neighbour change the other samples of its workgroup? (debug helper)"""
import dataclasses
import torch
from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused

pooled = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5)) for i, b in enumerate(DEFAULT_SPEC.blocks)))
single = dataclasses.replace(DEFAULT_SPEC, input_length=30, input_channels=1)
for name, spec in (("pooled", pooled), ("single30", single)):
    m = AlarconCNN1D(spec=spec, seed=5, device="cuda", params=R.synthetic_params(spec, 5))
    blob = m.fused_blob_x3()
    x0 = torch.randn(16, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(6)).cuda()
    for f in (1.0, 2.0, 3.0, 1e3, 1e-3):
        x = x0.clone()
        x[7] *= f
        full = fused.tiled_x3_forward(x, blob, spec, logits=True)[0, 0]
        singles = torch.stack([fused.tiled_x3_forward(x[i:i + 1], blob, spec, window_offset=i, logits=True)[0, 0, 0]
                               for i in range(16)])
        d = (singles - full).abs()
        print(name, "factor", f, "diff samples", (d > 0).nonzero().reshape(-1).tolist(), "max", float(d.max()))
