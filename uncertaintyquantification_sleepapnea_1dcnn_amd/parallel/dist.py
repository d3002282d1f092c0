"""Process-group setup: one process per GPU, ``torch.distributed`` over RCCL (backend "nccl").

The reference is single-process; distribution here is new.  Layout:

* ``world``: all ranks.  MC-Dropout shards *windows* over it (masks are keyed by global window
  index, so results are invariant to the GPU count).
* Deep Ensembles place members on ranks (``member_of_rank``); with more ranks than members the
  surplus ranks form data-parallel groups inside a member (``member_groups``), whose gradients
  are all-reduced (one fused bucket).

CPU tests use the ``gloo`` backend with the same code paths.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


_INFO: Optional[DistInfo] = None


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init(backend: Optional[str] = None, device: Optional[str] = None, timeout_s: int = 600) -> DistInfo:
    """Initialise from torchrun env vars (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*); no-op for one rank."""
    global _INFO
    if _INFO is not None:
        return _INFO
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = device != "cpu" and torch.cuda.is_available()
    # APNEAUQ_DIST_BACKEND=gloo rehearses a multi-rank GPU run on ONE card (RCCL refuses two ranks
    # on one device); production multi-GPU runs use RCCL ("nccl").  APNEAUQ_FORCE_PG=1 creates the
    # process group even for one rank (exercises the RCCL path on a 1-GPU box).
    force_pg = os.environ.get("APNEAUQ_FORCE_PG", "0") == "1"
    be = "none"
    if world > 1 or force_pg:
        be = backend or os.environ.get("APNEAUQ_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        n_dev = torch.cuda.device_count()
        if local >= n_dev and be != "gloo":
            raise RuntimeError(f"LOCAL_RANK {local} has no GPU ({n_dev} visible); one rank per GPU over RCCL")
        torch.cuda.set_device(local % max(1, n_dev))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if be != "none":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            from .launch import free_port

            os.environ["MASTER_PORT"] = str(free_port())
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if not dist.is_initialized():
            kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
    _INFO = DistInfo(rank, world, local, be, dev)
    return _INFO


def info() -> DistInfo:
    return _INFO if _INFO is not None else init()


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if info().backend == "nccl":
            dist.barrier(device_ids=[info().device.index])
        else:
            dist.barrier()


def shutdown() -> None:
    global _INFO
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None


def all_reduce_max(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=info().device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized():
        from . import comm

        comm.run("all_reduce", t, lambda: dist.all_reduce(t, op=dist.ReduceOp.SUM))
    return t


def shard_range(n: int, rank: int, world: int):
    """Contiguous [start, stop) block of n items for this rank (first ranks get the remainder)."""
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def members_of_rank(n_members: int, rank: int, world: int) -> List[int]:
    """Member ids hosted by ``rank`` (round-robin: member m on rank m % world)."""
    return [m for m in range(n_members) if m % world == rank]


def member_groups(n_members: int, world: int) -> List[List[int]]:
    """Ranks cooperating on each member when world > n_members (data parallel inside a member)."""
    if world <= n_members:
        return [[m % world] for m in range(n_members)]
    per = world // n_members
    return [list(range(m * per, (m + 1) * per)) for m in range(n_members)]


def gather_device_ids() -> List[str]:
    """``host:device`` of every rank, in rank order (reported by the benches)."""
    import socket

    me = f"{socket.gethostname()}:{info().device}"
    if not (dist.is_available() and dist.is_initialized()):
        return [me]
    out: List[Optional[str]] = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return [str(o) for o in out]
