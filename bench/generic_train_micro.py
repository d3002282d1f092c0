"""Micro-benchmark of one training step (forward + backward + Adam, batch-statistics BN) for
non-reference architectures on the generic HIP path (``ops/generic_train.py``) against the fp32
PyTorch autograd path those architectures used before, at the reference batch size (1024,
``cnn_baseline_train.py:29``).  ``reference`` runs the reference architecture through the generic
kernels for comparison with its dedicated kernels (``bench/train_micro.py``)."""
import argparse
import json
import os
import time

import torch

from bench.generic_micro import SPECS
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import generic_train
from uncertaintyquantification_sleepapnea_1dcnn_amd.training import step as tstep


def _time(fn, iters):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--specs", default="pooled,single30,reference")
    ap.add_argument("--no-torch", action="store_true", help="skip the fp32 autograd comparator")
    a = ap.parse_args()
    res = {}
    for name in a.specs.split(","):
        spec = SPECS[name]
        m = AlarconCNN1D(spec=spec, seed=1, device="cuda")
        x = torch.randn(a.batch, spec.input_length, spec.input_channels, device="cuda")
        y = (torch.rand(a.batch, device="cuda") > 0.5).float()
        eager = _time(lambda: generic_train.train_step(m, x, y), a.iters)
        hip = _time(lambda: generic_train.graph_train_step(m, x, y), a.iters)  # HIP-graph replay (the default path)
        r = {"hip_generic_ms": hip * 1e3, "hip_generic_eager_ms": eager * 1e3, "hip_windows_per_s": a.batch / hip,
             "train_tflops_eff": 3 * 2 * spec.forward_macs() * a.batch / hip / 1e12}
        if not a.no_torch:
            os.environ["APNEAUQ_TRAIN_BACKEND"] = "torch"
            try:
                tt = _time(lambda: tstep.train_step(m, x, y), max(3, a.iters // 4))
            finally:
                del os.environ["APNEAUQ_TRAIN_BACKEND"]
            r.update({"torch_fp32_ms": tt * 1e3, "speedup": tt / hip})
        res[name] = r
    print(json.dumps({"batch": a.batch, "results": res}, indent=1))


if __name__ == "__main__":
    main()
