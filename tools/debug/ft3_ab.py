"""Fused x3 kernel: save logits of a fixed input set (compare two builds bitwise)."""
import dataclasses, sys
import torch
from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused

pooled = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5)) for i, b in enumerate(DEFAULT_SPEC.blocks)))
single = dataclasses.replace(DEFAULT_SPEC, input_length=30, input_channels=1)
out = {}
for name, spec in (("pooled", pooled), ("single30", single)):
    m = AlarconCNN1D(spec=spec, seed=5, device="cuda", params=R.synthetic_params(spec, 5))
    blob = m.fused_blob_x3()
    x = torch.randn(333, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(6)).cuda()
    x[7] *= 1e3
    x[100] *= 1e-3
    for drop in (False, True):
        out[f"{name}_{drop}"] = fused.tiled_x3_forward(x, blob, spec, n_pass=3, dropout=drop, seed=1, logits=True).cpu()
torch.save(out, sys.argv[1])
