"""Host-side cost of replaying the graphed training step: which host calls between two replays of the
same graph wait for the previous replay to finish?  Prints median host microseconds per loop iteration
(no sync inside the loop) and the wall time per step."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, train_ops  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
m = AlarconCNN1D(seed=1, device="cuda")
g = torch.Generator().manual_seed(1)
x = torch.randn(batch, 60, 4, generator=g).cuda()
y = (torch.rand(batch, generator=g) < 0.3).float().cuda()
st = train_ops.GraphedTrainStep(m, batch)
for _ in range(10):
    st(x, y)
torch.cuda.synchronize()
o = _ext.ops()
ws = st.ws
side = torch.cuda.Stream()
z = torch.zeros(16, device="cuda")


def inputs():
    o.train_inputs([x], [y], [ws.x[train_ops.HALO:]], [ws.y], train_ops.SR)


variants = {
    "replay": lambda: st.graph.replay(),
    "replay + tiny torch op": lambda: (st.graph.replay(), z.add_(1.0)),
    "replay + train_inputs": lambda: (st.graph.replay(), inputs()),
    "train_inputs + replay": lambda: (inputs(), st.graph.replay()),
    "full call": lambda: st(x, y),
}
for label, fn in variants.items():
    ts = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(40):
        a = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    print(f"batch {batch} {label:24s}: host us/iter median {1e6 * statistics.median(ts):7.1f}; "
          f"wall us/iter {1e6 * tot / 40:7.1f}", flush=True)
