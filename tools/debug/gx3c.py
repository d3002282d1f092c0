"""Diagnostic: intermediate buffers of one fp32 train step, fp16x3 engine vs exact engine."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_fp32_gpu import ALL, _batch  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import generic_train  # noqa: E402

spec = ALL[sys.argv[1] if len(sys.argv) > 1 else "reference"]
bufs = {}
for eng in ("exact", "x3"):
    generic_train.FP32_ENGINE = eng
    m = AlarconCNN1D(spec=spec, seed=5, device="cuda", train_precision="fp32")
    x, y = _batch(spec, 64, 3)
    m.optimizer.learning_rate = 0.0
    generic_train.train_step(m, x, y)
    ws = m._gtrain_ws32
    d = {}
    for l in range(len(spec.blocks)):
        d[f"xin{l}"] = ws.xin[l].clone()
        d[f"z{l}"] = ws.z[l].clone()
        d[f"dzp{l}"] = ws.dzp[l].clone()
        d[f"dbs{l}"] = ws.dbs[l].clone()
        if ws.dh[l] is not None:
            d[f"dh{l}"] = ws.dh[l].clone()
        d[f"coef{l}"] = ws.coef[l].clone()
        d[f"bst{l}"] = ws.bst[l].clone()
        d[f"bn{l}"] = ws.bn[l].clone()
    bufs[eng] = d
for k in bufs["exact"]:
    a, b = bufs["exact"][k].double(), bufs["x3"][k].double()
    den = a.abs().max().item() or 1.0
    print(f"{k:8s} max|exact| {den:.3e}  max|diff|/max {((a - b).abs().max().item() / den):.2e}")

a, b = bufs["exact"]["dzp2"].double(), bufs["x3"]["dzp2"].double()
diff = (a - b).abs()
bad = (diff > 1e-5 * a.abs().max()).nonzero()
print("dzp2 shape", tuple(a.shape), "bad", len(bad), "rows", sorted(set(bad[:, 0].tolist()))[:40])
print("cols", sorted(set(bad[:, 1].tolist()))[:64])
r, c = bad[0].tolist()
print("sample", r, c, a[r, c].item(), b[r, c].item())
