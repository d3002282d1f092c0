"""GPU time per graphed training step when other work is enqueued between replays: a torch elementwise
op on the same / another stream, our own HIP kernel, and the real fit() loop (wall time per step)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, train_ops  # noqa: E402

batch = 1024
m = AlarconCNN1D(seed=1, device="cuda")
g = torch.Generator().manual_seed(1)
x = torch.randn(batch, 60, 4, generator=g).cuda()
y = (torch.rand(batch, generator=g) < 0.3).float().cuda()
for _ in range(5):
    m.train_step(x, y, return_probs=True)
torch.cuda.synchronize()
st = m._train_graphs[batch]
z = torch.zeros(16, device="cuda")
side = torch.cuda.Stream()


def side_op():
    with torch.cuda.stream(side):
        z.add_(1.0)


xs = torch.randn(8 * batch, 60, 4, generator=g).cuda()
idx = torch.randperm(8 * batch, device="cuda")[:batch]
variants = {
    "train_step": lambda: m.train_step(x, y, return_probs=True),
    "train_step + z.add_": lambda: (m.train_step(x, y, return_probs=True), z.add_(1.0)),
    "train_step + side-stream op": lambda: (m.train_step(x, y, return_probs=True), side_op()),
    "index_select + train_step": lambda: m.train_step(xs.index_select(0, idx), y, return_probs=True),
    "train_step + empty_cache-free alloc": lambda: (m.train_step(x, y, return_probs=True), torch.empty(16, device="cuda")),
}
for label, fn in variants.items():
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(40):
        fn()
    torch.cuda.synchronize()
    print(f"{label:36s}: wall us/step {1e6 * (time.perf_counter() - t0) / 40:8.1f}", flush=True)

n = 32 * batch
X = np.random.default_rng(0).standard_normal((n, 60, 4)).astype(np.float32)
Y = (np.random.default_rng(1).random(n) < 0.3).astype(np.float32)
m.fit(X[:2048], Y[:2048], batch_size=batch, epochs=1, verbose=0, shuffle=False)
torch.cuda.synchronize()
for shuffle in (False, True):
    t0 = time.perf_counter()
    m.fit(X, Y, batch_size=batch, epochs=1, verbose=0, shuffle=shuffle)
    torch.cuda.synchronize()
    print(f"fit 1 epoch x {n // batch} steps shuffle={shuffle}: wall us/step {1e6 * (time.perf_counter() - t0) / (n // batch):8.1f}",
          flush=True)
