"""Per-tensor relative gradient error: HIP training step vs bf16-dataflow emulation vs fp32 autograd."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tests.test_train_gpu import _torch_grads, _rel
from tests.train_emulation import emulate_step
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops
from uncertaintyquantification_sleepapnea_1dcnn_amd.training.step import TRAIN_PASS_BASE

for n in (64, 37):
    m = AlarconCNN1D(seed=5, device="cuda")
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, 60, 4, generator=g).cuda()
    y = (torch.rand(n, generator=g) > 0.5).float().cuda()
    m.optimizer.learning_rate = 0.0
    p0 = {k: v.clone() for k, v in m.store.as_dict().items()}
    rl, rg, rs, rlog = _torch_grads(m, x, y)
    el, elog, eg, est = emulate_step(m.spec, p0, x, y, m.seed, TRAIN_PASS_BASE)
    loss, _ = train_ops.train_step(m, x, y)
    ws = m._train_ws
    print(f"n={n} loss {loss.item():.5f} emu {el:.5f} ref {rl:.5f}  logits-vs-emu {(ws.logits[:n]-elog).abs().max().item():.2e}")
    for name in m.store.trainable:
        off, k = m.store.offsets[name], m.store.views[name].numel()
        a, b, e = ws.grad[off:off + k], rg[off:off + k], eg[name].reshape(-1)
        print(f"  {name:28s} hip-emu {_rel(a, e):.4f}  emu-ref {_rel(e, b):.4f}  hip-ref {_rel(a, b):.4f}")
