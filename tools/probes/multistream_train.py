"""Probe: M ensemble members' graphed HIP training steps on 1 GPU, sequential on one stream vs
round-robin over S HIP streams (kernels of different members run concurrently)."""
import json
import sys
import time

import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D


def run(models, x, y, streams, steps):
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        for i, m in enumerate(models):
            with torch.cuda.stream(streams[i % len(streams)]):
                m.train_step(x, y, return_probs=True)  # device tensors: no host sync per step
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    B = 1024
    dev = torch.device("cuda")
    models = [AlarconCNN1D(seed=100 + m, device=dev) for m in range(M)]
    x = torch.randn(B, 60, 4, device=dev)
    y = (torch.rand(B, device=dev) < 0.3).float()
    res = {}
    for S in (1, 2, 4, 8):
        streams = [torch.cuda.Stream() for _ in range(S)]
        run(models, x, y, streams, 3)  # warmup / graph capture
        dt = run(models, x, y, streams, 20)
        res[f"streams_{S}"] = {"ms_per_ensemble_step": round(dt * 1e3, 3), "windows_per_s": round(M * B / dt, 1)}
    print(json.dumps({"members": M, "batch": B, **res}))


if __name__ == "__main__":
    main()
