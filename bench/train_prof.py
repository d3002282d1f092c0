"""Short training-step loop for kernel traces (``rocprofv3 --kernel-trace --stats -- python -m
bench.train_prof --batch 1024 --steps 40``): the graphed single-model bf16 step (or fp32 with
``--fp32``) of the reference CNN on synthetic windows."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--fp32", action="store_true")
    a = ap.parse_args()
    import torch

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D

    g = torch.Generator().manual_seed(1)
    x = torch.randn(a.batch, 60, 4, generator=g).cuda()
    y = (torch.rand(a.batch, generator=g) < 0.3).float().cuda()
    m = AlarconCNN1D(seed=1, device="cuda", train_precision="fp32" if a.fp32 else "bf16")
    for _ in range(a.steps):
        m.train_step(x, y, return_probs=True)
    torch.cuda.synchronize()
    print("done", a.batch, a.steps)


if __name__ == "__main__":
    main()
