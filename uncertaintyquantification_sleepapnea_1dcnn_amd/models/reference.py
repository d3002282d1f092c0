"""Pure-PyTorch fp32 reference of the Alarcón 1D-CNN with exact Keras 2.12 semantics.

This is the numerics oracle for every HIP kernel (SURVEY §4 test pyramid, level 2) and the
CPU fallback used by the plumbing config "1D-CNN single forward on CPU".  It mirrors
``models/cnn_baseline_train.py:55-94``:

* channels-last input ``(N, L, C)``; ``Conv1D(padding='same')`` pads ``(k-1)//2`` left and
  ``k-1-(k-1)//2`` right; ReLU is *inside* the conv layer, i.e. **before** BatchNorm;
* BatchNormalization: eps 1e-3, momentum 0.99, biased batch variance for both the
  normalisation and the moving-average update (``tf.nn.moments``);
* inverted Dropout with the counter-based masks of :mod:`..ops.rng`;
* optional ``MaxPooling1D(2)`` (valid) after BN, before Dropout (reference blocks have it
  commented out, ``train_deep_ensemble_cnns.py:36-66``);
* ``GlobalAveragePooling1D`` then ``Dense(1, sigmoid)``.

Weights live in a dict keyed by the Keras names of :meth:`ModelSpec.weight_names`.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import rng
from .spec import ModelSpec

Params = Dict[str, torch.Tensor]


def glorot_uniform(shape, fan_in: int, fan_out: int, gen: torch.Generator) -> torch.Tensor:
    limit = math.sqrt(6.0 / float(fan_in + fan_out))
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2.0 - 1.0).mul_(limit).float()


def init_params(spec: ModelSpec, seed: int = 2025) -> Params:
    """Keras-default initialisation: glorot_uniform kernels, zero biases, BN (1, 0, 0, 1)."""
    gen = torch.Generator().manual_seed(int(seed))
    ch = spec.channels()
    p: Params = {}
    for i, b in enumerate(spec.blocks, start=1):
        k, cin, cout = b.kernel_size, ch[i - 1], b.filters
        # Keras conv fan_in = k*Cin, fan_out = k*Cout (receptive-field size times channels)
        p[f"conv1d_{i}/kernel"] = glorot_uniform((k, cin, cout), k * cin, k * cout, gen)
        p[f"conv1d_{i}/bias"] = torch.zeros(cout)
        p[f"batchnorm_{i}/gamma"] = torch.ones(cout)
        p[f"batchnorm_{i}/beta"] = torch.zeros(cout)
        p[f"batchnorm_{i}/moving_mean"] = torch.zeros(cout)
        p[f"batchnorm_{i}/moving_variance"] = torch.ones(cout)
    c = spec.final_channels
    p["output_layer/kernel"] = glorot_uniform((c, 1), c, 1, gen)
    p["output_layer/bias"] = torch.zeros(1)
    return p


def synthetic_params(spec: ModelSpec, seed: int = 2025) -> Params:
    """Random-init weights with non-trivial BN statistics (benchmarks: nothing folds to identity)."""
    p = init_params(spec, seed)
    g = torch.Generator().manual_seed(int(seed) + 7919)
    for i, b in enumerate(spec.blocks, start=1):
        c = b.filters
        p[f"batchnorm_{i}/moving_mean"] = torch.rand(c, generator=g) * 0.5
        p[f"batchnorm_{i}/moving_variance"] = torch.rand(c, generator=g) + 0.5
        p[f"batchnorm_{i}/gamma"] = torch.rand(c, generator=g) + 0.5
        p[f"batchnorm_{i}/beta"] = torch.randn(c, generator=g) * 0.1
    return p


def params_to_list(spec: ModelSpec, p: Params) -> List[np.ndarray]:
    return [p[n].detach().cpu().numpy().astype(np.float32) for n in spec.weight_names()]


def params_from_list(spec: ModelSpec, arrays, device=None) -> Params:
    names, shapes = spec.weight_names(), spec.weight_shapes()
    if len(arrays) != len(names):
        raise ValueError(f"expected {len(names)} weight arrays, got {len(arrays)}")
    out: Params = {}
    for n, s, a in zip(names, shapes, arrays):
        a = np.asarray(a, dtype=np.float32)
        if tuple(a.shape) != tuple(s):
            raise ValueError(f"{n}: expected shape {s}, got {a.shape}")
        out[n] = torch.from_numpy(a.copy()).to(device) if device is not None else torch.from_numpy(a.copy())
    return out


def conv1d_same(x: torch.Tensor, kernel: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """Keras Conv1D(padding='same') on channels-last x (N, L, Cin), kernel (k, Cin, Cout)."""
    k = kernel.shape[0]
    left = (k - 1) // 2
    right = k - 1 - left
    xt = F.pad(x.transpose(1, 2), (left, right))
    y = F.conv1d(xt, kernel.permute(2, 1, 0), bias)
    return y.transpose(1, 2)


def forward(
    spec: ModelSpec,
    p: Params,
    x: torch.Tensor,
    training: bool = False,
    *,
    dropout: Optional[bool] = None,
    bn_batch_stats: Optional[bool] = None,
    update_moving: bool = False,
    seed: int = 0,
    pass_id: int = 0,
    sample_ids: Optional[torch.Tensor] = None,
    return_logits: bool = False,
    bn_stats_hook=None,
    dtype: Optional[torch.dtype] = None,
    relu_masks=None,
) -> torch.Tensor:
    """Forward pass; returns probabilities (N, 1) (or logits).

    ``training=True`` matches Keras ``model(x, training=True)``: dropout on and BN on batch
    statistics.  ``dropout`` / ``bn_batch_stats`` override the two independently
    (``dropout=True, bn_batch_stats=False`` is standard MC Dropout, bn_mode="running").
    ``update_moving`` applies the Keras moving-average update in place (the side effect of
    the reference MC Dropout loop).  ``bn_stats_hook(h) -> (mean, var)`` replaces the
    local batch statistics (data-parallel SyncBN: global moments via a differentiable all-reduce).
    ``dtype`` (default fp32, the reference's precision) selects the compute dtype; tests use float64
    (with float64 parameters) as the exact oracle the fp32 paths are measured against.  ``relu_masks``
    (one bool (N, L, C) tensor per block) replaces each ReLU's branch choice by the given pattern -- the
    oracle then differentiates the same piecewise-linear branch as an fp32 run whose pre-activations
    sat within rounding of zero (a flipped ReLU moves a gradient by a whole element, not by rounding).
    """
    use_drop = training if dropout is None else dropout
    use_batch = training if bn_batch_stats is None else bn_batch_stats
    n = x.shape[0]
    if sample_ids is None:
        sample_ids = torch.arange(n, device=x.device)
    h = x.float() if dtype is None else x.to(dtype)
    for i, b in enumerate(spec.blocks, start=1):
        h = conv1d_same(h, p[f"conv1d_{i}/kernel"], p[f"conv1d_{i}/bias"])
        h = torch.relu(h) if relu_masks is None else h * relu_masks[i - 1].to(h.dtype)
        gamma, beta = p[f"batchnorm_{i}/gamma"], p[f"batchnorm_{i}/beta"]
        mm, mv = p[f"batchnorm_{i}/moving_mean"], p[f"batchnorm_{i}/moving_variance"]
        if use_batch:
            if bn_stats_hook is not None:
                mean, var = bn_stats_hook(h)
            else:
                mean = h.mean(dim=(0, 1))
                var = h.var(dim=(0, 1), unbiased=False)
            if update_moving:
                with torch.no_grad():
                    mm.mul_(spec.bn_momentum).add_(mean.detach() * (1 - spec.bn_momentum))
                    mv.mul_(spec.bn_momentum).add_(var.detach() * (1 - spec.bn_momentum))
        else:
            mean, var = mm, mv
        h = (h - mean) * torch.rsqrt(var + spec.bn_epsilon) * gamma + beta
        if b.pool:
            h = F.max_pool1d(h.transpose(1, 2), 2).transpose(1, 2)
        if use_drop and b.dropout > 0:
            key = rng.stream_key(seed, i - 1, pass_id)
            h = rng.dropout_apply_torch(h, key, sample_ids, b.dropout)
    g = h.mean(dim=1)
    logit = g @ p["output_layer/kernel"] + p["output_layer/bias"]
    return logit if return_logits else torch.sigmoid(logit)


def bn_fold(spec: ModelSpec, p: Params, i: int):
    """Inference BN of block i (1-based) as a per-channel affine (scale, shift)."""
    gamma, beta = p[f"batchnorm_{i}/gamma"], p[f"batchnorm_{i}/beta"]
    mm, mv = p[f"batchnorm_{i}/moving_mean"], p[f"batchnorm_{i}/moving_variance"]
    scale = gamma * torch.rsqrt(mv + spec.bn_epsilon)
    return scale, beta - mm * scale
