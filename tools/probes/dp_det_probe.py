"""Deterministic-mode DP (2 ranks on the box's GPU, gloo) vs 1 rank: gradient / stats deltas per tensor."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.dist_utils import run_ranks  # noqa: E402
from tests.test_deterministic_gpu import _data, _dp_step  # noqa: E402

if __name__ == "__main__":
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops

    os.environ["APNEAUQ_TRAIN_GRAPH"] = "0"
    res = run_ranks(_dp_step, 2, gpu=True)
    train_ops.set_deterministic(True)
    x, y = _data(128, 5)
    m = AlarconCNN1D(seed=3, device="cuda")
    m.train_step(x.cuda(), y.cuda())
    g1 = m._train_ws.grad.cpu()
    st = m.store
    flat, stats, grad = res[0]
    print("stats max abs diff", (stats - st.stats.cpu()).abs().max().item())
    for nm in st.trainable:
        off, k = st.offsets[nm], st.views[nm].numel()
        a, b = grad[off: off + k], g1[off: off + k]
        print(f"{nm:32s} |g|max {b.abs().max().item():.3e}  max|d| {(a - b).abs().max().item():.3e}  "
              f"rel-norm {((a - b).norm() / b.norm().clamp_min(1e-30)).item():.3e}")
