"""Multi-GPU UQ sampling behind the reference API (SURVEY §2.5 MC-sample / window / ensemble parallel).

The reference runs its 50 MC-Dropout passes and its ensemble members one after the other on one
device (``uq_techniques.py:22,29``).  Under ``torchrun`` (one process per GPU, RCCL over xGMI)
the same calls shard the work:

* **MC Dropout** — windows are split into contiguous shards, one per rank
  (``parallel.dist.shard_range``).  Dropout masks are keyed by the GLOBAL window index, so the
  samples are bitwise those of a single-GPU run.  ``bn_mode="running"``: every rank runs the fused
  kernel on its shard.  ``bn_mode="batch"`` (reference parity): the layer-synchronous batch-stat
  path with SyncBN (one all-reduce of the per-layer moment sums per pass chunk), so the
  statistics are those of the whole test set, exactly as the single-batch reference computes them.
* **Deep Ensemble** — member m runs on rank ``m % world`` (all windows; one fused launch for the
  rank's members).
* **Bootstrap**  — each rank reduces the per-window metrics of its window shard and
  sums the bootstrap draws that land in it; one all-reduce of the (B, 8) float64 raw sums gives
  every rank the replicate means (:func:`bootstrap_sharded`).
* Results are all-gathered so every rank returns the full (T|M, N, 1) array the
  reference API promises; the drivers then do host-side work on rank 0 only.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..parallel import dist as pdist


def active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _comm_device() -> torch.device:
    """RCCL moves device tensors; gloo (CPU tests, ranks sharing one GPU) gathers host tensors."""
    return torch.device("cpu") if dist.get_backend() == "gloo" else pdist.info().device


def _gather_windows(local: torch.Tensor, n_global: int, world: int) -> torch.Tensor:
    """(R, n_local) shards (contiguous, uneven by at most 1) -> (R, n_global) on every rank."""
    q = -(-n_global // world)
    pad = torch.zeros(local.shape[0], q, dtype=local.dtype, device=local.device)
    pad[:, :local.shape[1]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    parts = []
    for r in range(world):
        s, e = pdist.shard_range(n_global, r, world)
        parts.append(bufs[r][:, :e - s])
    return torch.cat(parts, dim=1)


def _gather_members(local: torch.Tensor, ids: List[int], n_members: int, world: int) -> torch.Tensor:
    """Rank-local (len(ids), N) member rows -> (M, N) on every rank (members round-robin)."""
    per = -(-n_members // world)
    pad = torch.zeros(per, local.shape[1], dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    out = torch.empty(n_members, local.shape[1], dtype=local.dtype, device=local.device)
    for r in range(world):
        mine = pdist.members_of_rank(n_members, r, world)
        out[mine] = bufs[r][:len(mine)]
    return out


@torch.no_grad()
def mc_dropout_predict_sharded(model, x_test_data, n_pred: int = 50, bn_mode: str = "batch",
                               seed: Optional[int] = None) -> torch.Tensor:
    """(T, N, 1) float32 on every rank; each rank computes its window shard."""
    from ..ops import bn_batch

    world, rank = dist.get_world_size(), dist.get_rank()
    x = model._as_input(x_test_data)
    n = x.shape[0]
    s, e = pdist.shard_range(n, rank, world)
    xl = x[s:e]
    seed = model.seed if seed is None else seed
    if bn_mode == "running":
        base = model._call_counter  # fresh masks per call, identical on every rank
        if model.uses_hip():
            loc = model.hip_infer(xl, n_pass=n_pred, dropout=True, seed=seed, window_offset=s, pass_offset=base)
        else:
            ids = torch.arange(s, e, device=x.device)
            loc = torch.stack([torch.sigmoid(model.logits(xl, dropout=True, bn_batch_stats=False, pass_id=base + t,
                                                          seed=seed, sample_ids=ids)).reshape(-1)
                               for t in range(n_pred)])
        model._call_counter = base + n_pred
    else:
        loc = bn_batch.mc_dropout_batch_bn(model, xl, n_pred, seed=seed, window_offset=s, distributed=True,
                                           global_n=n)[..., 0]
    comm = loc.float().to(_comm_device())
    return _gather_windows(comm, n, world).unsqueeze(-1)


@torch.no_grad()
def deep_ensembles_predict_sharded(ensemble_models: List, x_test_data) -> torch.Tensor:
    """(M, N, 1) float32 on every rank; member m is evaluated on rank m % world."""
    from ..ops import fused

    world, rank = dist.get_world_size(), dist.get_rank()
    M = len(ensemble_models)
    ids = pdist.members_of_rank(M, rank, world)
    dev = _comm_device()
    mine = [ensemble_models[i] for i in ids]
    if mine and all(m.uses_x3() for m in mine):
        from ..ops import x3

        m0 = mine[0]
        eng = x3.X3Model(m0.spec, [{k: v.to(m0.device) for k, v in m.store.as_dict().items()} for m in mine],
                         device=m0.device)
        loc = x3.forward_running(eng, m0._as_input(x_test_data))[:, 0]
    elif mine and all(m.uses_fused() for m in mine):
        x = mine[0]._as_input(x_test_data).to(torch.bfloat16).contiguous()
        blobs = torch.cat([m.fused_blob().to(mine[0].device) for m in mine])
        loc = fused.fused_forward(x, blobs, mine[0].spec)[:, 0]
    elif mine and all(m.uses_hip() for m in mine):
        x = mine[0]._as_input(x_test_data)
        loc = torch.stack([m.hip_infer(x)[0] for m in mine])
    elif mine:
        loc = torch.stack([torch.as_tensor(np.asarray(m.predict(x_test_data, verbose=0))).reshape(-1) for m in mine])
    else:
        n = np.asarray(x_test_data).shape[0] if not isinstance(x_test_data, torch.Tensor) else x_test_data.shape[0]
        loc = torch.zeros(0, n)
    return _gather_members(loc.float().to(dev), ids, M, world).unsqueeze(-1)


@torch.no_grad()
def bootstrap_sharded(predictions, y_true, n_boot: int, seed: int = 0, idx=None) -> torch.Tensor:
    """(B, 6) float64 bootstrap replicate means on every rank (``uq_techniques.py:137-157``).

    ``predictions`` is either the full (T, N) array (every rank slices its window shard) or this
    rank's (T, n_local) shard of the contiguous split ``shard_range(N, rank, world)`` — pass
    ``n_global`` via ``y_true`` being the full label vector in both cases.  ``idx`` (B, N)
    parity indices or the device counter hash (``seed``) pick the draws; the result equals the
    single-process ``ops.uq.bootstrap`` up to float64 summation order."""
    from ..ops import uq as uq_ops

    world, rank = dist.get_world_size(), dist.get_rank()
    y = torch.as_tensor(np.asarray(y_true.cpu() if isinstance(y_true, torch.Tensor) else y_true)).reshape(-1)
    n = y.numel()
    s, e = pdist.shard_range(n, rank, world)
    p = predictions if isinstance(predictions, torch.Tensor) else torch.as_tensor(np.asarray(predictions))
    if p.dim() == 3 and p.shape[-1] == 1:
        p = p[..., 0]
    if p.dim() == 1:
        p = p.reshape(1, -1)
    if p.shape[1] == n and e - s != n:
        p = p[:, s:e]
    assert p.shape[1] == e - s, (p.shape, s, e)
    dev = pdist.info().device if (torch.cuda.is_available() and dist.get_backend() != "gloo") else \
        (p.device if p.is_cuda else torch.device("cpu"))
    m = uq_ops.metrics(p.to(dev, torch.float32).contiguous())
    ii = None if idx is None else torch.as_tensor(np.asarray(idx.cpu() if isinstance(idx, torch.Tensor) else idx)
                                                  .astype(np.int32)).to(dev)
    part = uq_ops.bootstrap_partial(m, y[s:e].to(dev, torch.int32), n_boot, n, s, idx=ii, seed=seed)
    comm = part.to(_comm_device())
    dist.all_reduce(comm)
    return uq_ops.finalize_bootstrap_sums(comm, n)
