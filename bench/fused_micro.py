"""Micro-benchmark of the fused inference kernel (MC Dropout T passes / Deep Ensemble M members)."""
import argparse
import json
import time

import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as S
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--T", type=int, default=50)
    ap.add_argument("--M", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    x = torch.randn(a.n, 60, 4, device=dev).to(torch.bfloat16)
    blob1 = F.pack_blob(S, {k: v.to(dev) for k, v in R.init_params(S, 1).items()}).unsqueeze(0)
    blobs = torch.stack([F.pack_blob(S, {k: v.to(dev) for k, v in R.init_params(S, 10 + m).items()}) for m in range(a.M)])
    res = {}
    for name, fn, samples in [
        ("mcd", lambda: F.fused_forward(x, blob1, S, n_pass=a.T, dropout=True, seed=7), a.n * a.T),
        ("de", lambda: F.fused_forward(x, blobs, S), a.n * a.M),
        ("det", lambda: F.fused_forward(x, blob1, S), a.n),
    ]:
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        flops = samples * 2 * S.forward_macs() * 64 / 60
        res[name] = {"ms": dt * 1e3, "samples_per_s": samples / dt, "windows_per_s": a.n / dt,
                     "tflops_eff": samples * 2 * S.forward_macs() / dt / 1e12, "tflops_issued": flops / dt / 1e12}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
