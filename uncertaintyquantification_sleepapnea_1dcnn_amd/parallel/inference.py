"""Multi-GPU UQ inference: window-sharded MC Dropout and member-parallel Deep Ensembles.

Replaces the reference's serial loops (``uq_techniques.py:22`` over T passes, ``:29`` over M
members, both on one device) with:

* **MC Dropout** — windows sharded contiguously over ranks; every rank runs all T passes of its
  shard in ONE fused launch (``ops/fused.py``).  Dropout masks are keyed by the global window
  index, so the (T, N) probabilities do not depend on the GPU count.
* **Deep Ensemble** — member-parallel: rank r hosts members ``[r*M/G, (r+1)*M/G)`` and runs them
  over the whole (resident) window set; one RCCL ``all_to_all`` over xGMI then hands every rank
  the M member probabilities of its own window shard, where the entropy / MI
  reduction runs.  Falls back to replicated members + window sharding when G does not divide M.
* Aggregates (sums for the 6 UQ scalars + counts) are combined with one small all-reduce (C4).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..models.spec import DEFAULT_SPEC, ModelSpec
from ..ops import fused, uq as uq_ops
from . import dist as pdist


def mcd_probs_local(blob: torch.Tensor, x_local_bf16: torch.Tensor, n_pass: int, seed: int, window_offset: int,
                    spec: ModelSpec = DEFAULT_SPEC) -> torch.Tensor:
    """(T, N_local) MC-Dropout probabilities of this rank's window shard."""
    return fused.fused_forward(x_local_bf16, blob, spec, n_pass=n_pass, dropout=True, seed=seed,
                               window_offset=window_offset)[0]


def all_to_all_members(p_local: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """(M/G, N_global) member probabilities of this rank's members over ALL windows ->
    (M, N_global/G) probabilities of ALL members over this rank's window shard (one RCCL all_to_all)."""
    if world == 1:
        return p_local
    mloc, ng = p_local.shape
    n = ng // world
    send = p_local.reshape(mloc, world, n).transpose(0, 1).contiguous()  # (G dest, M/G, n)
    recv = torch.empty_like(send)  # (G src, M/G, n)
    from . import comm

    if send.is_cuda and dist.get_backend(group) == "gloo":  # single-card rehearsal: gloo has no GPU all_to_all
        rc = recv.cpu()
        sc = send.cpu()
        comm.run("all_to_all", sc, lambda: dist.all_to_all_single(rc, sc, group=group))
        recv.copy_(rc)
    else:
        comm.run("all_to_all", send, lambda: dist.all_to_all_single(recv, send, group=group))
    return recv.reshape(world * mloc, n)


def de_probs_member_parallel(blobs_local: torch.Tensor, x_global_bf16: torch.Tensor, world: int,
                             spec: ModelSpec = DEFAULT_SPEC, group=None) -> torch.Tensor:
    """(M, N_global/G) ensemble probabilities of this rank's window shard.

    ``blobs_local``: (M/G, bytes) members hosted here; ``x_global_bf16``: (N_global, 60, 4)
    resident on every rank, N_global divisible by G.
    """
    p = fused.fused_forward(x_global_bf16, blobs_local, spec)[:, 0]  # (M/G, N_global)
    return all_to_all_members(p, world, group)


def aggregate_sums(metrics: torch.Tensor, y: Optional[torch.Tensor]) -> torch.Tensor:
    """Per-rank partial sums for the 6 scalar UQ aggregates: returns (9,) float64.

    [n, sum var, sum var|y=0, n0, sum var|y=1, n1, sum H, sum E[H], sum MI]
    """
    var = metrics[uq_ops.VAR].double()
    out = torch.zeros(9, dtype=torch.float64, device=metrics.device)
    out[0] = metrics.shape[1]
    out[1] = var.sum()
    if y is not None:
        m0 = (y == 0)
        m1 = (y == 1)
        out[2] = (var * m0).sum()
        out[3] = m0.sum()
        out[4] = (var * m1).sum()
        out[5] = m1.sum()
    out[6] = metrics[uq_ops.ENT_NATS].double().sum()
    out[7] = metrics[uq_ops.EXP_ENT].double().sum()
    out[8] = metrics[uq_ops.MI].double().sum()
    return out


def finalize_aggregates(s: torch.Tensor) -> Dict[str, float]:
    s = s.detach().cpu().tolist()
    n = max(s[0], 1.0)
    return {
        "overall_mean_variance": s[1] / n,
        "mean_variance_class_0": s[2] / s[3] if s[3] > 0 else 0.0,
        "mean_variance_class_1": s[4] / s[5] if s[5] > 0 else 0.0,
        "mean_total_pred_entropy": s[6] / n,
        "mean_expected_aleatoric_entropy": s[7] / n,
        "mean_mutual_info": s[8] / n,
    }


def global_aggregates(metrics: torch.Tensor, y: Optional[torch.Tensor]) -> Tuple[torch.Tensor, Dict[str, float]]:
    s = aggregate_sums(metrics, y)
    pdist.all_reduce_sum_(s)
    return s, finalize_aggregates(s)
