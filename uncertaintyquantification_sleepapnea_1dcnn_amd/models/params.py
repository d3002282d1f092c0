"""Flat parameter storage.

All trainable tensors of a model live in ONE contiguous fp32 buffer (``flat``) and the BN moving
statistics in a second one (``stats``); the Keras-named tensors are views into them.  This gives
the multi-tensor Adam kernel a single launch over 851,457 values and the data-parallel gradient
all-reduce a single fused bucket, and makes ``get_weights`` / restore-best /
member checkpoints cheap copies.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch

from .spec import ModelSpec


class ParamStore:
    def __init__(self, spec: ModelSpec, params: Dict[str, torch.Tensor], device=None):
        self.spec = spec
        names, shapes, train = spec.weight_names(), spec.weight_shapes(), spec.trainable_mask()
        dev = torch.device(device) if device is not None else params[names[0]].device
        self.names = names
        self.shapes = {n: tuple(s) for n, s in zip(names, shapes)}
        self.trainable = [n for n, t in zip(names, train) if t]
        self.nontrainable = [n for n, t in zip(names, train) if not t]
        nt = sum(int(np.prod(self.shapes[n])) for n in self.trainable)
        ns = sum(int(np.prod(self.shapes[n])) for n in self.nontrainable)
        self.flat = torch.zeros(nt, dtype=torch.float32, device=dev)
        self.stats = torch.zeros(ns, dtype=torch.float32, device=dev)
        self.views: Dict[str, torch.Tensor] = {}
        self.offsets: Dict[str, int] = {}
        off = 0
        for n in self.trainable:
            k = int(np.prod(self.shapes[n]))
            self.views[n] = self.flat[off: off + k].view(self.shapes[n])
            self.offsets[n] = off
            off += k
        off = 0
        for n in self.nontrainable:
            k = int(np.prod(self.shapes[n]))
            self.views[n] = self.stats[off: off + k].view(self.shapes[n])
            off += k
        with torch.no_grad():
            for n in names:
                self.views[n].copy_(params[n].to(dev).float().reshape(self.shapes[n]))
        self.version = 0

    @property
    def device(self):
        return self.flat.device

    def as_dict(self) -> Dict[str, torch.Tensor]:
        return dict(self.views)

    def bump(self) -> None:
        self.version += 1

    def get_weights(self) -> List[np.ndarray]:
        return [self.views[n].detach().cpu().numpy().copy() for n in self.names]

    def set_weights(self, arrays) -> None:
        if len(arrays) != len(self.names):
            raise ValueError(f"expected {len(self.names)} arrays, got {len(arrays)}")
        with torch.no_grad():
            for n, a in zip(self.names, arrays):
                a = np.asarray(a, dtype=np.float32)
                if tuple(a.shape) != self.shapes[n]:
                    raise ValueError(f"{n}: expected {self.shapes[n]}, got {a.shape}")
                self.views[n].copy_(torch.from_numpy(a).to(self.device))
        self.bump()

    def snapshot(self):
        return self.flat.detach().clone(), self.stats.detach().clone()

    def restore(self, snap) -> None:
        with torch.no_grad():
            self.flat.copy_(snap[0])
            self.stats.copy_(snap[1])
        self.bump()

    def to(self, device) -> "ParamStore":
        return ParamStore(self.spec, self.as_dict(), device)
