"""Diagnostic: per-tensor gradient deviation of the fp16x3 fp32 engine vs the exact fp32 engine and the
float64 oracle on one spec (python tools/debug_gx3.py [spec])."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_fp32_gpu import ALL, _batch, _grads64  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import generic_train  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "reference"
spec = ALL[name]
res = {}
for eng in ("exact", "x3"):
    generic_train.FP32_ENGINE = eng
    m = AlarconCNN1D(spec=spec, seed=5, device="cuda", train_precision="fp32")
    x, y = _batch(spec, 64, 3)
    m.optimizer.learning_rate = 0.0
    if eng == "exact":
        ref_loss, ref_grad, _ = _grads64(m, x, y)
    loss, _ = generic_train.train_step(m, x, y)
    res[eng] = (loss.item(), m._gtrain_ws32.grad.clone(), m)
st = res["x3"][2].store
print("loss", ref_loss, {k: v[0] for k, v in res.items()})
for nm in st.trainable:
    off, k = st.offsets[nm], st.views[nm].numel()
    r = ref_grad[off: off + k]
    print(f"{nm:28s} |ref| {r.norm().item():.3e}  exact {((res['exact'][1][off:off+k]-r).norm()/r.norm()).item():.2e}"
          f"  x3 {((res['x3'][1][off:off+k]-r).norm()/r.norm()).item():.2e}")
