"""Data parallelism inside one ensemble member (used when there are more GPUs than members).

A member's global batch (1024, ``cnn_baseline_train.py:28``) is split contiguously over the ranks
of its group.  Equivalence with single-device Keras training is exact up to reduction order:

* every rank draws the same epoch permutation (same seed) and takes its contiguous slice;
* dropout masks are keyed by the sample's position in the *global* batch (``window_offset``);
* BatchNorm uses global moments: the per-channel sums (forward) and the backward sums are
  all-reduced between layers (SyncBN) — the HIP path all-reduces the kernels' moment
  buffers, the autograd path uses a differentiable all-reduce;
* the loss is the global-batch mean, so summing the ranks' gradients (one flat bucket, C1) gives
  the single-device gradient.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DPContext:
    group: Optional[object]
    size: int
    rank: int

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def moments_hook(self):
        """Differentiable SyncBN moments for the autograd path: h -> (mean, var) over the group."""
        from torch.distributed.nn.functional import all_reduce as dall_reduce

        grp = self.group

        def hook(h: torch.Tensor):
            s1 = h.sum(dim=(0, 1))
            s2 = (h * h).sum(dim=(0, 1))
            n = torch.tensor([float(h.shape[0] * h.shape[1])], device=h.device)
            buf = torch.cat([s1, s2, n])
            buf = dall_reduce(buf, group=grp) if self.size > 1 else buf
            c = s1.numel()
            mean = buf[:c] / buf[2 * c]
            var = buf[c: 2 * c] / buf[2 * c] - mean * mean
            return mean, var.clamp_min(0)

        return hook


def split_batch(idx: torch.Tensor, dp: Optional[DPContext]):
    """Local slice of a global batch index vector and its offset within the global batch."""
    if dp is None or dp.size == 1:
        return idx, 0
    parts = torch.tensor_split(idx, dp.size)
    off = sum(int(p.numel()) for p in parts[: dp.rank])
    return parts[dp.rank], off
