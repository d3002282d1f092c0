"""Eager vs eager vs graph losses of the generic training step (nondeterminism calibration)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_generic_gpu import SPECS  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402

for name in ("pooled", "single30"):
    spec = SPECS[name]
    g = torch.Generator().manual_seed(3)
    x = torch.randn(256, spec.input_length, spec.input_channels, generator=g).cuda()
    y = (torch.rand(256, generator=g) < 0.4).float().cuda()
    for mode in ("0", "0", "1", "1"):
        os.environ["APNEAUQ_TRAIN_GRAPH"] = mode
        m = AlarconCNN1D(spec=spec, seed=4, device="cuda")
        losses = [round(float(m.train_step(x[i * 64:(i + 1) * 64], y[i * 64:(i + 1) * 64])), 4) for i in range(4)]
        print(name, mode, losses, flush=True)
