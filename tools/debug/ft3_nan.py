"""Fused x3 kernel with NaN-filled LDS (probe build): which outputs read uninitialised LDS?"""
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
    x = torch.randn(16, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(6)).cuda()
    for drop in (False, True):
        y = fused.tiled_x3_forward(x, blob, spec, n_pass=2, dropout=drop, seed=1, logits=True)[0]
        ref = R.forward(spec, {k: v.double() for k, v in R.synthetic_params(spec, 5).items()}, x.double().cpu(),
                        dropout=drop, seed=1, pass_id=0, return_logits=True, dtype=torch.float64).reshape(-1)
        print(name, drop, "nan outputs", int(torch.isnan(y).sum()), "max err pass0", float((y[0].double().cpu() - ref).abs().max()))
