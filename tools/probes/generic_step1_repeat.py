"""Repeatability of the generic (pooled) training step 1 loss: eager and graph, fresh models."""
import collections
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_generic_gpu import SPECS  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402

spec = SPECS["pooled"]
g = torch.Generator().manual_seed(3)
x = torch.randn(256, spec.input_length, spec.input_channels, generator=g).cuda()
y = (torch.rand(256, generator=g) < 0.4).float().cuda()
for mode in ("0", "1"):
    os.environ["APNEAUQ_TRAIN_GRAPH"] = mode
    seen = collections.Counter()
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):  # noqa: B007
        m = AlarconCNN1D(spec=spec, seed=4, device="cuda")
        seen[round(float(m.train_step(x[:64], y[:64])), 4)] += 1
        del m
        gc.collect()
    print(mode, dict(seen), flush=True)
