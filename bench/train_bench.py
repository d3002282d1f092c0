"""Deep-Ensemble training throughput (BASELINE.json config "DE M=8 training across 8 x MI355X").

Ensemble parallel as in ``parallel/ensemble.py``: member m trains on rank m % G (one process per GPU,
``torchrun --nproc-per-node G``), every member runs Keras-semantics steps (batch 1024, Adam,
BCE, dropout, batch-statistics BN) on synthetic SHHS2-shaped windows through the HIP training
kernels.  One "step" = one optimizer step of EVERY member; windows/s counts all members' samples
over all GPUs (weak scaling in members per GPU when G | M).

    python -m bench.train_bench --members 8 --steps 20             # 1 GPU, members on 3 streams
    python -m bench.train_bench --gpus 8 --members 8               # self-launches 8 ranks (one per GPU)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m bench.train_bench --gpus 8 --members 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); self-launched unless under torchrun")
    ap.add_argument("--members", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--streams", type=int, default=3, help="HIP streams the members of one GPU round-robin over "
                    "(3 + the default stream fit the 4 hardware queues HIP uses per process; --mode streams)")
    ap.add_argument("--groups", type=int, default=4, help="batched mode: member groups, one batched graph each, "
                    "replayed on their own HIP streams (4: the best of 1/2/3/4/8 for 8 members)")
    ap.add_argument("--mode", choices=["batched", "streams"], default="batched",
                    help="batched: one member-batched HIP graph per step (ops/train_ops.py:GraphedEnsembleStep); "
                         "streams: members' graphs overlapped on HIP streams")
    a = ap.parse_args(argv)
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import launch

    rc = launch.maybe_spawn(a.gpus, __file__, argv)  # before anything touches the GPU
    if rc is not None:
        sys.exit(rc)
    import torch

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import dist as pdist

    launch.check_world(a.gpus, int(os.environ.get("WORLD_SIZE", "1")), torch.cuda.device_count())
    info = pdist.init()
    dev = info.device
    mine = pdist.members_of_rank(a.members, info.rank, info.world)
    models = [AlarconCNN1D(seed=a.seed + m, device=dev) for m in mine]
    g = torch.Generator().manual_seed(a.seed + info.rank)
    x = torch.randn(a.batch, 60, 4, generator=g).to(dev)
    y = (torch.rand(a.batch, generator=g) < 0.3).float().to(dev)

    # members sharing a GPU overlap on separate streams (a batch-1024 step fills only part of the
    # GPU); train_step(return_probs=True) returns device tensors, so nothing syncs per step
    streams = [torch.cuda.Stream(device=dev) for _ in range(max(1, min(a.streams, len(models))))]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream(dev))

    batched = a.mode == "batched" and len(models) > 1
    if batched:
        from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops

        ng = max(1, min(a.groups, len(models)))
        parts = [models[i::ng] for i in range(ng)]
        ens = [train_ops.GraphedEnsembleStep(p, a.batch) for p in parts]
        gstreams = [torch.cuda.Stream(device=dev) for _ in parts] if ng > 1 else [None]
        for s_ in gstreams:
            if s_ is not None:
                s_.wait_stream(torch.cuda.current_stream(dev))

    def step():
        if batched:
            for e, p, s_ in zip(ens, parts, gstreams):
                if s_ is None:
                    e([x] * len(p), [y] * len(p))
                else:
                    with torch.cuda.stream(s_):
                        e([x] * len(p), [y] * len(p))
            return
        for i, mdl in enumerate(models):
            with torch.cuda.stream(streams[i % len(streams)]):
                mdl.train_step(x, y, return_probs=True)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    pdist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    pdist.barrier()
    dt = pdist.all_reduce_max(time.perf_counter() - t0)
    devices = pdist.gather_device_ids()
    if info.rank == 0:
        samples = a.members * a.batch * a.steps
        print(json.dumps({"metric": "DE training windows/s (all members, all GPUs)", "value": round(samples / dt, 1),
                          "n_gpus": info.world, "members": a.members, "batch": a.batch, "steps": a.steps,
                          "ms_per_step_all_members": round(dt * 1e3 / a.steps, 3), "dtype": "bf16",
                          "data": "synthetic", "backend": info.backend, "devices": devices,
                          "parallelism": f"ensemble-parallel over {info.world} GPU(s), " +
                          (f"member-batched launches ({len(parts)} group(s))" if batched else f"{len(streams)} stream(s)/GPU")}))
    pdist.shutdown()


if __name__ == "__main__":
    main()
