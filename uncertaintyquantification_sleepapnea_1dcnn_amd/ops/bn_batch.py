"""MC Dropout with BatchNorm on batch statistics — exact reference semantics.

The reference's ``mc_dropout_predict`` calls ``model(x_test, training=True)`` T times with the
WHOLE test set as one batch (``uq_techniques.py:22``): dropout on, every BN layer normalises with
the mean / biased variance of that pass's activations over all windows, and the moving averages
are updated as a side effect (momentum 0.99, once per pass and layer).  Statistics are global over
the test set, so execution is layer-synchronous: block l of every window must finish before block
l+1 of any window can be normalised.

``mc_dropout_batch_bn`` reproduces this.  With several GPUs the per-layer moments are combined
with an all-reduce of (sum, sum of squares, count) per channel so that the result
equals the single-device full-batch computation.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..models import reference as R


def _moments_hook(group=None):
    import torch.distributed as dist

    def hook(h: torch.Tensor):
        s1 = h.sum(dim=(0, 1), dtype=torch.float64)
        s2 = (h.double() * h.double()).sum(dim=(0, 1))
        cnt = torch.tensor([h.shape[0] * h.shape[1]], dtype=torch.float64, device=h.device)
        if dist.is_available() and dist.is_initialized():
            buf = torch.cat([s1, s2, cnt])
            dist.all_reduce(buf, group=group)
            c = s1.numel()
            s1, s2, cnt = buf[:c], buf[c: 2 * c], buf[2 * c:]
        mean = s1 / cnt
        var = (s2 / cnt - mean * mean).clamp_min(0)
        return mean.float(), var.float()

    return hook


@torch.no_grad()
def mc_dropout_batch_bn(model, x, n_pred: int, seed: Optional[int] = None, window_offset: int = 0,
                        distributed: bool = False, update_moving: bool = True, global_n: Optional[int] = None,
                        chunk_rows: Optional[int] = None) -> torch.Tensor:
    """(T, N, 1) probabilities; each pass = Keras ``model(x, training=True)`` on the full set.

    On a GPU with the HIP extension: the fp32-faithful engine for the reference architecture
    (``x3.mcd_batch``, precision "fp32", the default), else the bf16 layer-wise training kernels
    (``train_ops`` / ``generic_train.forward_batch_stats``); BN moments accumulated in the conv
    epilogue, SyncBN by one all-reduce per layer when ``distributed``.  Otherwise the fp32 PyTorch
    reference path.  ``global_n`` = windows over all ranks; ``chunk_rows`` (ranks must
    agree on it) bounds the windows x passes processed per launch.
    """
    xt = model._as_input(x)
    n = xt.shape[0]
    if xt.is_cuda and getattr(model, "uses_x3", lambda: False)():
        # fp32-faithful engine (the reference's precision); window-chunked beyond the memory budget
        from . import x3

        sync = None
        if distributed:
            import torch.distributed as dist

            if dist.is_available() and dist.is_initialized():
                sync = dist.all_reduce
        base = model._call_counter
        out = x3.mcd_batch(model.x3_model(), xt, n_pred, seed=model.seed if seed is None else seed, pass_base=base,
                           window_offset=window_offset, update_moving=update_moving, sync=sync, global_n=global_n,
                           max_samples=chunk_rows)
        model._call_counter = base + n_pred
        if update_moving:
            model.store.bump()  # the moving statistics were updated in place
        return out.unsqueeze(-1)
    if xt.is_cuda:
        from . import train_ops

        if train_ops.supports(model.spec):
            sync = None
            if distributed:
                import torch.distributed as dist

                if dist.is_available() and dist.is_initialized():
                    sync = dist.all_reduce
            base = model._call_counter
            out = train_ops.forward_batch_stats(model, xt, n_pred, pass_base=base, seed=model.seed if seed is None else seed,
                                                update_moving=update_moving, sync=sync, window_offset=window_offset,
                                                global_n=global_n, max_samples=chunk_rows or (1 << 20))
            model._call_counter = base + n_pred
            return out.unsqueeze(-1)
        from . import generic_train

        if generic_train.supports(model.spec):
            sync = None
            if distributed:
                import torch.distributed as dist

                if dist.is_available() and dist.is_initialized():
                    sync = dist.all_reduce
            base = model._call_counter
            out = generic_train.forward_batch_stats(model, xt, n_pred, pass_base=base,
                                                    seed=model.seed if seed is None else seed,
                                                    update_moving=update_moving, sync=sync,
                                                    window_offset=window_offset, global_n=global_n)
            model._call_counter = base + n_pred
            return out.unsqueeze(-1)
        from . import fused

        fused.warn_unsupported(model.spec, "batch-statistics MC Dropout")
    sample_ids = torch.arange(window_offset, window_offset + n, device=xt.device)
    hook = _moments_hook() if distributed else None
    outs = []
    base = model._call_counter
    for t in range(n_pred):
        logit = R.forward(model.spec, model.store.as_dict(), xt, dropout=True, bn_batch_stats=True,
                          update_moving=update_moving, seed=model.seed if seed is None else seed,
                          pass_id=base + t, sample_ids=sample_ids, return_logits=True, bn_stats_hook=hook)
        outs.append(torch.sigmoid(logit))
    model._call_counter = base + n_pred
    if update_moving:
        model.store.bump()
    return torch.stack(outs)
