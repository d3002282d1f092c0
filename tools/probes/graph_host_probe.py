"""Where does model.train_step spend host time between graph replays (batch 1024)?  Host us per call
(median, no sync in the loop) and wall us per step for the layers of the call chain."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.training import step as tstep  # noqa: E402

batch = 1024
m = AlarconCNN1D(seed=1, device="cuda")
g = torch.Generator().manual_seed(1)
x = torch.randn(batch, 60, 4, generator=g).cuda()
y = (torch.rand(batch, generator=g) < 0.3).float().cuda()
for _ in range(5):
    m.train_step(x, y, return_probs=True)
torch.cuda.synchronize()
st = m._train_graphs[batch]


def step_call():
    r = st(x, y)
    m._train_step_counter += 1
    return r


def graph_fn():
    r = train_ops.graph_train_step(m, x, y)
    m._train_step_counter += 1
    return r


def tstep_fn():
    r = tstep.train_step(m, x, y)
    m._train_step_counter += 1
    return r


variants = {"replay": lambda: st.graph.replay(), "GraphedTrainStep.__call__": step_call,
            "graph_train_step": graph_fn, "training.step.train_step": tstep_fn,
            "model.train_step": lambda: m.train_step(x, y, return_probs=True)}
for rep in range(2):
    for label, fn in variants.items():
        ts = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(40):
            a = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - a)
        torch.cuda.synchronize()
        print(f"{label:28s}: host us/call median {1e6 * statistics.median(ts):7.1f}; wall us/step "
              f"{1e6 * (time.perf_counter() - t0) / 40:7.1f}", flush=True)
