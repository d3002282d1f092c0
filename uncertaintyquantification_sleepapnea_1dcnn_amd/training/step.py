"""One Keras-semantics optimizer step (forward in training mode, BCE-on-logits, backward, Adam).

Backends:
* ``"hip"``  — the reference architecture's layer-wise HIP kernels (``ops/train_ops.py``);
* ``"hip_generic"`` — any other architecture (pool blocks, other window shapes) on the generic
  HIP kernels (``ops/generic_train.py``), and every architecture with ``train_precision="fp32"``
  (fp32 activations / gradients, fp32-input MFMA convs, ``csrc/gf32_conv.hip``);
* ``"torch"``— autograd over the fp32 reference ops (CPU, and the fallback/oracle on GPU).

Gradients land in ONE flat fp32 buffer (views of ``ParamStore.flat``), so the data-parallel
all-reduce is a single bucket and Adam is a single launch.
"""
from __future__ import annotations

import os

import torch

from ..models import reference as R

TRAIN_PASS_BASE = 1 << 30  # dropout pass ids used by training steps (disjoint from MC-Dropout passes)


def _backend(model) -> str:
    b = os.environ.get("APNEAUQ_TRAIN_BACKEND", "auto")
    if b != "auto":
        return b
    if model.device.type == "cuda":
        from ..ops import generic_train, train_ops

        if getattr(model, "train_precision", "bf16") == "fp32":  # any architecture, fp32 kernels
            if generic_train.supports_fp32(model.spec):
                return "hip_generic"
        elif train_ops.supports(model.spec):
            return "hip"
        elif generic_train.supports(model.spec):
            return "hip_generic"
        from ..ops import fused

        fused.warn_unsupported(model.spec, "training")
    return "torch"


def _use_graphs() -> bool:
    """HIP-graph replay of the single-device HIP step (``APNEAUQ_TRAIN_GRAPH=0`` disables)."""
    return os.environ.get("APNEAUQ_TRAIN_GRAPH", "1") != "0"


def train_step(model, x: torch.Tensor, y: torch.Tensor, grad_allreduce=None, dp_step=None):
    """``dp_step = (global_batch, offset)`` when the model trains data-parallel (``model.dp``)."""
    backend = _backend(model)
    dp = getattr(model, "dp", None)
    if dp is not None and dp.size == 1:
        dp = None
    gn, off = dp_step if (dp is not None and dp_step is not None) else (x.shape[0], 0)
    if backend == "hip_generic":
        from ..ops import generic_train

        if dp is not None:
            return generic_train.train_step(model, x, y, grad_allreduce=lambda g: (dp.all_reduce_(g), 1.0)[1],
                                            sync=dp.all_reduce_, global_batch=gn, window_offset=off,
                                            sync_world=dp.size)
        if grad_allreduce is None and _use_graphs():
            return generic_train.graph_train_step(model, x, y)
        return generic_train.train_step(model, x, y, grad_allreduce=grad_allreduce)
    if backend == "hip":
        from ..ops import train_ops

        if dp is not None:
            def _gar(g):
                dp.all_reduce_(g)
                return 1.0  # kernels already scale by 1/global batch

            return train_ops.train_step(model, x, y, grad_allreduce=_gar, sync=dp.all_reduce_, global_batch=gn,
                                        window_offset=off, sync_world=dp.size)
        if grad_allreduce is None and _use_graphs():
            return train_ops.graph_train_step(model, x, y)
        return train_ops.train_step(model, x, y, grad_allreduce=grad_allreduce)
    store = model.store
    flat = store.flat.detach().requires_grad_(True)
    p = {}
    for n in store.trainable:
        o = store.offsets[n]
        p[n] = flat[o: o + store.views[n].numel()].view(store.shapes[n])
    for n in store.nontrainable:
        p[n] = store.views[n]
    sample_ids = off + torch.arange(x.shape[0], device=x.device)
    logits = R.forward(model.spec, p, x, dropout=True, bn_batch_stats=True, update_moving=True, seed=model.seed,
                       pass_id=TRAIN_PASS_BASE + model._train_step_counter, sample_ids=sample_ids,
                       return_logits=True, bn_stats_hook=dp.moments_hook() if dp is not None else None)
    lv = torch.nn.functional.binary_cross_entropy_with_logits(logits.reshape(-1), y.reshape(-1), reduction="none")
    loss = lv.sum() / gn  # mean over the (global) batch
    loss.backward()
    grad = flat.grad
    scale = 1.0
    if dp is not None:
        dp.all_reduce_(grad)
    elif grad_allreduce is not None:
        scale = grad_allreduce(grad)
    model.optimizer.step(store.flat, grad, grad_scale=scale)
    return lv.detach().sum().double(), torch.sigmoid(logits.detach()).reshape(-1)
