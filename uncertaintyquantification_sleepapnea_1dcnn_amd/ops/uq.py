"""Device UQ reductions (``csrc/uq_reduce.hip``) with a bit-compatible eager fallback.

``metrics(probs)`` returns a (7, N) fp32 tensor whose rows are
[mean, variance(ddof=0), H(mean) nats, E[H] nats, MI, H(mean) bits(+1e-9), label(mean>0.5)] —
the per-window quantities of ``uq_techniques.py:62-91`` and ``analyze_mcd_patient_level.py:107-117``.
``bootstrap(metrics, y, B, idx|seed)`` returns (B, 6) float64 replicate aggregates.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _ext

MEAN, VAR, ENT_NATS, EXP_ENT, MI, ENT_BITS, LABEL = range(7)
ROW_NAMES = ("mean_pred", "pred_variance", "total_pred_entropy", "expected_aleatoric_entropy", "mutual_info",
             "entropy_bits", "label")


def _bin_entropy_nats_t(p: torch.Tensor) -> torch.Tensor:
    q = 1.0 - p
    p = p.clamp(1e-10, 1.0)
    q = q.clamp(1e-10, 1.0)
    s = p + q
    p, q = p / s, q / s
    return -(p * torch.log(p) + q * torch.log(q))


def metrics_eager(probs: torch.Tensor) -> torch.Tensor:
    p = probs.float()
    mean = p.mean(0)
    var = ((p - mean) ** 2).mean(0)
    h = _bin_entropy_nats_t(mean)
    e = _bin_entropy_nats_t(p).mean(0)
    bits = -(mean * torch.log2(mean + 1e-9) + (1 - mean) * torch.log2(1 - mean + 1e-9))
    return torch.stack([mean, var, h, e, (h - e).clamp_min(0), bits, (mean > 0.5).float()])


def metrics(probs: torch.Tensor) -> torch.Tensor:
    """(T, N) -> (7, N) per-window metrics; HIP kernel on the GPU."""
    if probs.dim() == 3:
        probs = probs.reshape(-1, probs.shape[-1])
    if probs.is_cuda:
        return _ext.ops().uq_reduce(probs.float().contiguous())
    return metrics_eager(probs)


def _hash_idx(n: int, n_boot: int, seed: int, device) -> torch.Tensor:
    from .rng import _mix32_t

    b = torch.arange(n_boot, device=device, dtype=torch.int64)[:, None]
    j = torch.arange(n, device=device, dtype=torch.int64)[None, :]
    bkey = _mix32_t(torch.full_like(b, seed & 0xFFFFFFFF) ^ _mix32_t((b * 0x9E3779B9 + 0x7F4A7C15) & 0xFFFFFFFF))
    h = _mix32_t(bkey ^ _mix32_t(j))
    return (h * n) >> 32


def bootstrap_eager(m: torch.Tensor, y: torch.Tensor, idx: Optional[torch.Tensor], seed: int, n_boot: int) -> torch.Tensor:
    n = m.shape[1]
    if idx is None:
        idx = _hash_idx(n, n_boot, seed, m.device)
    idx = idx.long()
    var, h, e, mi = m[VAR].double(), m[ENT_NATS].double(), m[EXP_ENT].double(), m[MI].double()
    yy = y.long()
    out = torch.zeros(n_boot, 6, dtype=torch.float64, device=m.device)
    for b in range(n_boot):
        ix = idx[b]
        v, yb = var[ix], yy[ix]
        out[b, 0] = v.mean()
        c0, c1 = (yb == 0), (yb == 1)
        out[b, 1] = v[c0].mean() if c0.any() else 0.0
        out[b, 2] = v[c1].mean() if c1.any() else 0.0
        out[b, 3] = h[ix].mean()
        out[b, 4] = e[ix].mean()
        out[b, 5] = mi[ix].mean()
    return out


def bootstrap(m: torch.Tensor, y: torch.Tensor, n_boot: int, idx: Optional[torch.Tensor] = None, seed: int = 0) -> torch.Tensor:
    """(B, 6) float64 bootstrap replicate aggregates (order = metrics.AGG_KEYS)."""
    if m.is_cuda:
        return _ext.ops().bootstrap(m, y.to(m.device), None if idx is None else idx.to(m.device), int(seed) & 0xFFFFFFFF,
                                    int(n_boot))
    return bootstrap_eager(m, y, idx, seed, n_boot)


def bootstrap_partial_eager(m_loc: torch.Tensor, y_loc: torch.Tensor, idx: Optional[torch.Tensor], seed: int,
                            n_boot: int, n_global: int, lo: int) -> torch.Tensor:
    """(B, 8) float64 raw sums over the draws that land in windows [lo, lo + n_loc): [sum var,
    sum var|y=0, n0, sum var|y=1, n1, sum H, sum E[H], sum MI] (bootstrap_kernel<true>)."""
    n_loc = m_loc.shape[1]
    if idx is None:
        idx = _hash_idx(n_global, n_boot, seed, m_loc.device)
    k = idx.long() - lo
    inside = (k >= 0) & (k < n_loc)
    var, h, e, mi = (m_loc[r].double() for r in (VAR, ENT_NATS, EXP_ENT, MI))
    yy = y_loc.long()
    out = torch.zeros(n_boot, 8, dtype=torch.float64, device=m_loc.device)
    for b in range(n_boot):
        kk = k[b][inside[b]]
        v, yb = var[kk], yy[kk]
        c0, c1 = yb == 0, yb == 1
        out[b] = torch.stack([v.sum(), v[c0].sum(), c0.sum().double(), v[c1].sum(), c1.sum().double(), h[kk].sum(),
                              e[kk].sum(), mi[kk].sum()])
    return out


def bootstrap_partial(m_loc: torch.Tensor, y_loc: torch.Tensor, n_boot: int, n_global: int, lo: int,
                      idx: Optional[torch.Tensor] = None, seed: int = 0) -> torch.Tensor:
    """This shard's (B, 8) bootstrap sums (HIP kernel on the GPU); sum them over ranks, then
    :func:`finalize_bootstrap_sums`."""
    if m_loc.is_cuda:
        return _ext.ops().bootstrap_partial(m_loc, y_loc.to(m_loc.device), None if idx is None else idx.to(m_loc.device),
                                            int(seed) & 0xFFFFFFFF, int(n_boot), int(n_global), int(lo))
    return bootstrap_partial_eager(m_loc, y_loc, idx, int(seed) & 0xFFFFFFFF, n_boot, n_global, lo)


def finalize_bootstrap_sums(s: torch.Tensor, n_global: int) -> torch.Tensor:
    """(B, 8) summed raw sums -> (B, 6) replicate means (order = metrics.AGG_KEYS)."""
    s = s.double()
    out = torch.zeros(s.shape[0], 6, dtype=torch.float64, device=s.device)
    out[:, 0] = s[:, 0] / n_global
    out[:, 1] = torch.where(s[:, 2] > 0, s[:, 1] / s[:, 2].clamp_min(1), torch.zeros_like(s[:, 1]))
    out[:, 2] = torch.where(s[:, 4] > 0, s[:, 3] / s[:, 4].clamp_min(1), torch.zeros_like(s[:, 3]))
    out[:, 3] = s[:, 5] / n_global
    out[:, 4] = s[:, 6] / n_global
    out[:, 5] = s[:, 7] / n_global
    return out
