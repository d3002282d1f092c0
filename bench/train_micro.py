"""Training-step throughput of the HIP training kernels (batch 1024, Keras semantics)."""
import argparse
import json
import time

import numpy as np
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--precision", default="bf16", help="train_precision (fp32: the fp32 kernels, backend auto)")
    a = ap.parse_args()
    import os
    os.environ["APNEAUQ_TRAIN_BACKEND"] = "auto" if a.precision == "fp32" else a.backend
    m = AlarconCNN1D(seed=1, device="cuda", train_precision=a.precision)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.batch, 60, 4, generator=g).cuda()
    y = (torch.rand(a.batch, generator=g) > 0.5).float().cuda()
    for _ in range(3):
        m.train_step(x, y)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        m.train_step(x, y, return_probs=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.steps
    print(json.dumps({"backend": a.backend, "precision": a.precision, "batch": a.batch, "ms_per_step": dt * 1e3, "windows_per_s": a.batch / dt,
                      "tflops_eff": 3 * 2 * 50.9e6 * a.batch / dt / 1e12}))


if __name__ == "__main__":
    main()
