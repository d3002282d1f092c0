"""Throughput of the user-facing Keras-style training loop (``model.fit``), the reference's
``fit(epochs=30, batch_size=1024, validation_split=0.1)`` (``cnn_baseline_train.py:210-217``),
on synthetic SHHS2-shaped windows: windows/s over whole epochs including shuffling, the graphed
HIP train step, the device-side K10 accuracy/AUC counters, and validation."""
from __future__ import annotations

import argparse
import json
import time

import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--n", type=int, default=131072)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--epochs", type=int, default=3)
    a = ap.parse_args(argv)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.n, 60, 4, generator=g)
    y = (x[:, :, 0].mean(1) > 0).float()
    m = AlarconCNN1D(seed=1, device="cuda")
    xd, yd = x.cuda(), y.cuda()
    m.fit(xd[: 4 * a.batch], yd[: 4 * a.batch], batch_size=a.batch, epochs=1, verbose=0)  # capture / warm up
    torch.cuda.synchronize()
    t = time.perf_counter()
    h = m.fit(xd, yd, batch_size=a.batch, epochs=a.epochs, verbose=0, validation_split=0.1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    n_train = a.n - int(a.n * 0.1)
    print(json.dumps({"metric": "fit windows/s (train windows per epoch / epoch time, incl. validation)",
                      "windows_per_s": n_train * a.epochs / dt, "s_per_epoch": dt / a.epochs,
                      "batch": a.batch, "n": a.n, "epochs": a.epochs,
                      "final": {k: v[-1] for k, v in h.history.items()}}))


if __name__ == "__main__":
    main()
