"""Which samples of the fused x3 kernel change with the workgroup composition (debug helper)."""
import dataclasses
import torch
from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused

spec = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5)) for i, b in enumerate(DEFAULT_SPEC.blocks)))
m = AlarconCNN1D(spec=spec, seed=5, device="cuda", params=R.synthetic_params(spec, 5))
x = torch.randn(45, 60, 4, generator=torch.Generator().manual_seed(6)).cuda()
x[7] *= 1e3
blob = m.fused_blob_x3()
for drop in (False, True):
    f1 = fused.tiled_x3_forward(x, blob, spec, n_pass=3, dropout=drop, seed=2, logits=True)[0]
    f2 = fused.tiled_x3_forward(x, blob, spec, n_pass=3, dropout=drop, seed=2, logits=True)[0]
    print("drop", drop, "repeat identical:", torch.equal(f1, f2))
    for cuts in (((0, 5), (5, 22), (22, 45)), ((0, 1), (1, 45)), ((0, 44), (44, 45))):
        parts = torch.cat([fused.tiled_x3_forward(x[a:b], blob, spec, n_pass=3, dropout=drop, seed=2, window_offset=a,
                                                  logits=True)[0] for a, b in cuts], dim=1)
        d = (parts - f1).abs()
        idx = (d > 0).nonzero().tolist()
        print("  cuts", cuts, "n diff", len(idx), "max", float(d.max()), idx[:10])
    # single-sample launches
    singles = torch.stack([fused.tiled_x3_forward(x[i:i + 1], blob, spec, n_pass=1, dropout=drop, seed=2, window_offset=i,
                                                  logits=True)[0, 0, 0] for i in range(45)])
    d = (singles - f1[0]).abs()
    print("  singles vs full pass0: n diff", int((d > 0).sum()), "max", float(d.max()), (d > 0).nonzero().reshape(-1).tolist()[:20])
