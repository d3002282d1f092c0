"""Speed of the fp32 precision paths beside their bf16 counterparts.

``python -m bench.fp32_micro``: one JSON line; ``measure()`` is also ``bench.py``'s ``extra.fp32_paths``.

* inference of the pooled ensemble architecture (``/root/reference/models/train_deep_ensemble_cnns.py:36-66``
  MaxPool variant, loaded by ``evaluate_de_global.py:18-38``): Deep-Ensemble predict of 8 members and
  batch-BN / running-BN MC Dropout (T = 50) over 16384 windows, ``precision="fp32"`` (the fused fp16x3
  kernel ``csrc/fused_tiled_x3.hip`` for DE / running BN, the fp16x3 layer-wise kernels for batch BN) vs
  ``"bf16"`` (fused / generic bf16 kernels);
* one training step (batch 1024, Keras semantics, HIP graph) of the reference CNN and of the pooled CNN,
  ``train_precision="fp32"`` (``ops/generic_train.py`` fp16x3 kernels) vs ``"bf16"``.

Random-init weights, synthetic (60, 4) windows; best of ``reps`` timings after one warm-up call.  Always
the single-device path (``distributed=False``): under ``torchrun`` ``bench.py`` calls it on rank 0 only,
between barriers, so the numbers are the fused kernels' own and carry no collectives.
"""
import argparse
import dataclasses
import json
import time

import numpy as np
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

POOLED = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                        for i, b in enumerate(DEFAULT_SPEC.blocks)))


def _best(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return round(min(ts), 3)


def measure(windows: int = 16384, members: int = 8, passes: int = 50, reps: int = 3, steps: int = 50,
            precisions=("fp32", "bf16")) -> dict:
    g = torch.Generator().manual_seed(0)
    x = torch.randn(windows, 60, 4, generator=g)
    xd = x.cuda()
    out = {"windows": windows, "members": members, "passes": passes, "pooled": {}, "train_b1024": {}}
    for prec in precisions:
        ms = [AlarconCNN1D(spec=POOLED, seed=10 + i, device="cuda", precision=prec) for i in range(members)]
        r = {"de_ms": _best(lambda: U.deep_ensembles_predict(ms, xd, as_numpy=False, distributed=False), reps),
             "mcd_batch_ms": _best(lambda: U.mc_dropout_predict(ms[0], xd, n_pred=passes, bn_mode="batch", seed=1,
                                                               as_numpy=False, distributed=False), reps),
             "mcd_running_ms": _best(lambda: U.mc_dropout_predict(ms[0], xd, n_pred=passes, bn_mode="running",
                                                                 seed=1, as_numpy=False, distributed=False), reps)}
        out["pooled"][prec] = r
        del ms
    xb = torch.randn(1024, 60, 4, generator=g).cuda()
    yb = (torch.rand(1024, generator=g) > 0.5).float().cuda()
    for name, spec in (("reference", DEFAULT_SPEC), ("pooled", POOLED)):
        for prec in precisions:
            m = AlarconCNN1D(spec=spec, seed=3, device="cuda", train_precision=prec)

            def run():
                for _ in range(steps):
                    m.train_step(xb, yb)

            t = _best(run, reps) / steps
            out["train_b1024"][f"{name}_{prec}"] = {"ms_per_step": round(t, 4),
                                                    "windows_per_s": round(1024 / t * 1e3, 1)}
            del m
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=16384)
    ap.add_argument("--members", type=int, default=8)
    ap.add_argument("--passes", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    print(json.dumps(measure(a.windows, a.members, a.passes, a.reps, a.steps)))


if __name__ == "__main__":
    main()
