"""Diagnostic: which launch modifies a buffer it should not (fp16x3 fp32 train step)."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_fp32_gpu import ALL, _batch  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, generic_train  # noqa: E402

spec = ALL["reference"]
generic_train.FP32_ENGINE = "x3"
m = AlarconCNN1D(spec=spec, seed=5, device="cuda", train_precision="fp32")
x, y = _batch(spec, 64, 3)
m.optimizer.learning_rate = 0.0
generic_train.train_step(m, x, y)  # allocate the workspace
ws = m._gtrain_ws32
real = _ext.ops()
watch = {f"dzp{l}": ws.dzp[l] for l in range(6)}
watch.update({f"dh{l}": ws.dh[l] for l in range(1, 6)})


class Spy:
    def __getattr__(self, name):
        f = getattr(real, name)

        def g(*a, **k):
            before = {n: t.clone() for n, t in watch.items()}
            r = f(*a, **k)
            torch.cuda.synchronize()
            ch = [n for n, t in watch.items() if not torch.equal(before[n], t)]
            print(name, "changed:", ch)
            return r
        return g


for t in watch.values():
    t.zero_()
_ext.ops = lambda: Spy()
generic_train.train_step(m, x, y)
