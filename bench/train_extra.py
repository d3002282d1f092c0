"""Training throughput block of ``bench.py`` (``extra.train``): BASELINE.json config #2, "training (Adam,
BCE) on 1 x MI355X".

The reference's training loop is Keras ``fit(batch_size=1024)`` with Adam and BCE
(``/root/reference/models/cnn_baseline_train.py:100-102,210-217``) and the sequential Deep-Ensemble
member loop (``/root/reference/models/train_deep_ensemble_cnns.py:125-177``).  Measured here, on the
HIP training kernels (``ops/train_ops.py``, ``csrc/train_conv.hip``), each step a complete optimizer
step (forward with batch-statistics BN and dropout, BCE, backward, Adam) of random-init weights on
synthetic (60, 4) windows:

* ``single_b1024``: one model, the graphed step at the reference's batch size;
* ``single_b8192``: one model at batch 8192 (the per-step work of 8 members);
* ``members8_b1024``: 8 ensemble members, each at batch 1024, as member-batched graphs
  (``GraphedEnsembleStep``, the trainer's groups (2 of 4) on their own HIP streams: ``training/trainer.py:_fit_batched``);
* ``loss_parity``: the same 10 steps (same init, batches, dropout masks) on the HIP kernels and on the
  fp32 PyTorch autograd step (``training/step.py`` backend "torch"): per-step relative loss deviation.
"""
from __future__ import annotations

import os
import time
from typing import Optional


def _timeit(torch, fn, steps: int, warmup: int) -> float:
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def measure(dev, seed: int = 2025, steps: int = 50, warmup: int = 5, members: int = 8, groups: Optional[int] = None,
            batch: int = 1024, big_batch: int = 8192, parity_steps: int = 10) -> dict:
    import torch

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops

    g = torch.Generator().manual_seed(seed)
    n = max(big_batch, batch * parity_steps)
    x = torch.randn(n, 60, 4, generator=g).to(dev)
    y = (torch.rand(n, generator=g) < 0.3).float().to(dev)
    out = {"semantics": "Keras train step: batch-stat BN + dropout forward, BCE on logits, backward, Adam "
                        "(lr 1e-3); bf16 MFMA operands, fp32 accumulation / master weights / BN moments (fp64)",
           "mode": "atomic (production) reductions, HIP-graph replay"}

    xb, yb = x[:batch], y[:batch]
    m = AlarconCNN1D(seed=seed, device=dev)
    t = _timeit(torch, lambda: m.train_step(xb, yb, return_probs=True), steps, warmup)
    out["single_b1024"] = {"batch": batch, "ms_per_step": round(t * 1e3, 4), "windows_per_s": round(batch / t, 1)}

    xl, yl = x[:big_batch], y[:big_batch]
    m8 = AlarconCNN1D(seed=seed + 1, device=dev)
    k = max(10, steps // 4)
    t = _timeit(torch, lambda: m8.train_step(xl, yl, return_probs=True), k, 3)
    out["single_b8192"] = {"batch": big_batch, "ms_per_step": round(t * 1e3, 4), "windows_per_s": round(big_batch / t, 1)}

    ms = [AlarconCNN1D(seed=seed + 10 + i, device=dev) for i in range(members)]
    if groups is None:  # the trainer's member-batched grouping (training/trainer.py:ENSEMBLE_GROUPS)
        from uncertaintyquantification_sleepapnea_1dcnn_amd.training.trainer import ENSEMBLE_GROUPS as groups
    ng = max(1, min(groups, members))
    parts = [list(range(members))[i::ng] for i in range(ng)]
    ens = [train_ops.GraphedEnsembleStep([ms[i] for i in p], batch) for p in parts]
    streams = [torch.cuda.Stream(device=dev) for _ in parts]
    cur = torch.cuda.current_stream(dev)
    xs = [x[(i % 8) * batch:(i % 8 + 1) * batch] for i in range(members)]
    ys = [y[(i % 8) * batch:(i % 8 + 1) * batch] for i in range(members)]

    for s_ in streams:  # the inputs were written on the default stream
        s_.wait_stream(cur)

    def ens_step():
        # each group's steps are ordered on its own stream; the groups are independent models, so (as in
        # training/trainer.py:_fit_batched) nothing joins them between steps (_timeit synchronizes the device)
        for p, st, s_ in zip(parts, ens, streams):
            with torch.cuda.stream(s_):
                st([xs[i] for i in p], [ys[i] for i in p])

    t = _timeit(torch, ens_step, steps, warmup)
    out["members8_b1024"] = {"members": members, "groups": ng, "batch_per_member": batch,
                             "ms_per_step": round(t * 1e3, 4), "windows_per_s": round(members * batch / t, 1)}

    # loss parity: the same steps on the HIP kernels and on fp32 autograd (backend "torch")
    losses = {}
    old = os.environ.get("APNEAUQ_TRAIN_BACKEND")
    try:
        for backend in ("hip", "torch"):
            os.environ["APNEAUQ_TRAIN_BACKEND"] = backend
            mp = AlarconCNN1D(seed=seed + 99, device=dev)
            losses[backend] = [mp.train_step(x[i * batch:(i + 1) * batch], y[i * batch:(i + 1) * batch]) / batch
                               for i in range(parity_steps)]
    finally:
        if old is None:
            os.environ.pop("APNEAUQ_TRAIN_BACKEND", None)
        else:
            os.environ["APNEAUQ_TRAIN_BACKEND"] = old
    rel = [abs(a - b) / abs(b) for a, b in zip(losses["hip"], losses["torch"])]
    out["loss_parity"] = {"steps": parity_steps, "batch": batch, "step1_rel": float(f"{rel[0]:.3e}"),
                          "max_rel": float(f"{max(rel):.3e}"),
                          "loss_hip": [round(v, 6) for v in losses["hip"]],
                          "loss_fp32_torch": [round(v, 6) for v in losses["torch"]]}
    return out
