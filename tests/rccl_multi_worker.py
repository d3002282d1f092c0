"""One rank of the multi-GPU RCCL checks (tests/test_rccl_multi_gpu.py), started by
``parallel.launch.spawn``: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* come from the environment, one
GPU per rank, backend "nccl" (= RCCL over xGMI).  Rank 0 writes one JSON line to $APNEAUQ_RESULT.

Checks (each against the same computation on ONE rank, done by rank 0 itself):
  * batch-BN MC Dropout, fp32-faithful engine, windows sharded + SyncBN all-reduce per layer
    (the reference's model(x, training=True) over the WHOLE window set, uq_techniques.py:22);
  * Deep-Ensemble member-parallel inference + all_to_all of member probabilities (uq_techniques.py:29);
  * one deterministic data-parallel training step (SyncBN + one gradient bucket).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import x3  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import dist as pdist  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import inference as pinf  # noqa: E402


def gather_rows(t: torch.Tensor, counts):
    """All-gather (T, n_r) shards of uneven width into (T, sum n_r) (pad to the widest)."""
    w = max(counts)
    pad = torch.zeros(t.shape[0], w, dtype=t.dtype, device=t.device)
    pad[:, : t.shape[1]] = t
    bufs = [torch.empty_like(pad) for _ in counts]
    dist.all_gather(bufs, pad)
    return torch.cat([b[:, :c] for b, c in zip(bufs, counts)], 1)


def main():
    info = pdist.init()
    rehearsal = os.environ.get("APNEAUQ_DIST_BACKEND") == "gloo"  # ranks sharing one GPU (logic check only)
    assert info.backend == ("gloo" if rehearsal else "nccl"), info.backend
    dev, rank, world = info.device, info.rank, info.world
    out = {"world": world, "backend": dist.get_backend(), "device": str(dev)}
    names = [None] * world
    dist.all_gather_object(names, str(torch.cuda.current_device()))
    out["devices"] = names

    # ---- batch-BN MC Dropout, windows sharded (uneven: 101 windows), SyncBN over the ranks
    n_glob, T, seed = 101, 3, 2025
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n_glob, 60, 4, generator=g)
    s0, s1 = pdist.shard_range(n_glob, rank, world)
    p = {k: v.to(dev) for k, v in R.synthetic_params(SPEC, 13).items()}
    m = x3.X3Model(SPEC, [p])
    ph = x3.mcd_batch(m, x[s0:s1].to(dev), T, seed=seed, pass_base=5, window_offset=s0, update_moving=True,
                      sync=lambda t: dist.all_reduce(t), global_n=n_glob)
    counts = [pdist.shard_range(n_glob, r, world)[1] - pdist.shard_range(n_glob, r, world)[0] for r in range(world)]
    full = gather_rows(ph, counts)
    # ---- Deep Ensemble: 2 members per rank over ALL windows, all_to_all to window shards
    M, n_de = 2 * world, 8 * world
    xd = torch.randn(n_de, 60, 4, generator=torch.Generator().manual_seed(9)).to(dev)
    mine = list(range(rank * 2, rank * 2 + 2))
    pm = [{k: v.to(dev) for k, v in R.synthetic_params(SPEC, 100 + i).items()} for i in mine]
    p_local = x3.forward_running(x3.X3Model(SPEC, pm), xd)[:, 0]          # (2, n_de)
    p_shard = pinf.all_to_all_members(p_local, world)                       # (M, n_de / world)
    de_full = gather_rows(p_shard, [n_de // world] * world)                 # (M, n_de)

    # ---- deterministic data-parallel training step (SyncBN + one gradient bucket)
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel.data_parallel import DPContext, split_batch

    os.environ["APNEAUQ_TRAIN_GRAPH"] = "0"
    train_ops.set_deterministic(True)
    gx = torch.Generator().manual_seed(5)
    xt = torch.randn(128, 60, 4, generator=gx)
    yt = (torch.rand(128, generator=gx) > 0.5).float()
    md = AlarconCNN1D(seed=3, device=dev)
    md.dp = DPContext(None, world, rank)
    idx, off = split_batch(torch.arange(128), md.dp)
    md.train_step(xt[idx].to(dev), yt[idx].to(dev), dp_step=(128, off))
    grad_dp = md._train_ws.grad.clone()
    stats_dp = md.store.stats.clone()
    flats = [torch.empty_like(md.store.flat) for _ in range(world)]
    dist.all_gather(flats, md.store.flat)

    if rank == 0:
        # the same three computations on this one rank
        p1 = {k: v.to(dev) for k, v in R.synthetic_params(SPEC, 13).items()}
        ref = x3.mcd_batch(x3.X3Model(SPEC, [p1]), x.to(dev), T, seed=seed, pass_base=5, update_moving=True)
        out["mcd_max_abs_dp"] = float((full - ref).abs().max())
        out["mcd_moving_stats_max_abs"] = max(float((p[k] - p1[k]).abs().max()) for k in p if "moving" in k)
        pa = [{k: v.to(dev) for k, v in R.synthetic_params(SPEC, 100 + i).items()} for i in range(M)]
        de_ref = x3.forward_running(x3.X3Model(SPEC, pa), xd)[:, 0]
        out["de_bitwise"] = bool(torch.equal(de_full, de_ref))
        out["de_max_abs_dp"] = float((de_full - de_ref).abs().max())
        m1 = AlarconCNN1D(seed=3, device=dev)
        m1.train_step(xt.to(dev), yt.to(dev))
        out["dp_grad_max_abs"] = float((grad_dp - m1._train_ws.grad).abs().max())
        out["dp_stats_max_abs"] = float((stats_dp - m1.store.stats).abs().max())
        out["dp_ranks_bitwise_equal"] = all(bool(torch.equal(f, flats[0])) for f in flats)
        with open(os.environ["APNEAUQ_RESULT"], "w") as f:
            f.write(json.dumps(out) + "\n")
    pdist.barrier()
    pdist.shutdown()


if __name__ == "__main__":
    main()
