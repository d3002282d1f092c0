#!/usr/bin/env python3
"""Headline benchmark: 30s-windows/sec for MC Dropout T=50 & Deep Ensemble M=8 UQ inference.

Driver contract (one rank per GPU; ``torchrun --nproc-per-node N bench.py --gpus N ...``):
one *step* processes a fixed batch of ``--windows`` windows PER GPU (weak scaling) through the
complete UQ inference of both methods the reference evaluates
(``uncertainty_quantification/analyze_mcd_patient_level.py`` / ``analyze_de_patient_level.py``):

  1. MC Dropout, T=50 stochastic passes (fused HIP kernel, counter-based dropout masks, BN on
     running statistics = standard MC Dropout) over this rank's window shard, then the per-window
     mean / variance / entropy / expected entropy / MI reduction (HIP ``uq_reduce``);
  2. Deep Ensemble, M=8 members (inference BN, no dropout) placed member-parallel over the GPUs,
     RCCL all_to_all of member probabilities over xGMI, then the same reduction;
  3. the 6 aggregate UQ scalars of each method, all-reduced over ranks.

``value`` = windows fully UQ-evaluated (both methods) per second over ALL GPUs.  Model: the
reference Alarcón 1D-CNN (853,441 params, 60 x 4 windows), random-init weights with non-trivial
BN statistics, synthetic standardised windows.  Timing: W untimed warmup steps, then K steps
bracketed by barrier + synchronize; the max over ranks is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused, uq as uq_ops  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import dist as pdist  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import inference as pinf  # noqa: E402

METRIC = "30s-windows/sec for MCD T=50 & DE M=8 inference at 1/2/4/8 MI355X"
# The reference publishes no throughput number.  vs_baseline divides by OUR
# measurement of its exact loops in eager fp32 PyTorch on 1 x MI355X (bench/comparator.py, N=16384,
# MCD T=50 with BN batch statistics as the reference runs it + DE M=8 predict(batch 32) + NumPy UQ
# metrics): profiles/comparator_eager_fp32_batchbn_r1.json.  It is the faster of the two comparator
# modes (BN running statistics: 3102 windows/s), so the ratio is the conservative one.
BASELINE = 4925.9


def synthetic_params(seed: int):
    return R.synthetic_params(SPEC, seed)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--windows", type=int, default=16384, help="windows per GPU per step")
    ap.add_argument("--passes", type=int, default=50, help="MC Dropout passes T")
    ap.add_argument("--members", type=int, default=8, help="Deep Ensemble members M")
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--bn-mode", choices=["running", "batch"], default="running",
                    help="MC-Dropout BatchNorm: running statistics (standard MC Dropout, fused kernel) or "
                         "per-pass batch statistics over the whole window set = the reference's "
                         "model(x, training=True) (layer-wise HIP kernels + SyncBN across ranks)")
    a = ap.parse_args(argv)

    info = pdist.init()
    dev = info.device
    if dev.type != "cuda":
        raise SystemExit("bench.py needs a GPU")
    world, rank = info.world, info.rank
    n_loc = a.windows
    n_glob = n_loc * world

    # ---- resident data: the whole synthetic window set lives in HBM on every rank (bf16)
    g = torch.Generator(device="cpu").manual_seed(a.seed)
    x_glob = torch.randn(n_glob, 60, 4, generator=g).to(torch.bfloat16).to(dev)
    y_glob = (torch.rand(n_glob, generator=g) < 0.3).to(torch.int32).to(dev)
    start, stop = pdist.shard_range(n_glob, rank, world)
    x_loc = x_glob[start:stop].contiguous()
    y_loc = y_glob[start:stop].contiguous()

    # ---- models: one MC-Dropout model; M ensemble members, member-parallel when G | M
    blob_mcd = fused.pack_blob(SPEC, {k: v.to(dev) for k, v in synthetic_params(a.seed).items()}).unsqueeze(0)
    member_parallel = world > 1 and a.members % world == 0
    mem_ids = (list(range(rank * (a.members // world), (rank + 1) * (a.members // world)))
               if member_parallel else list(range(a.members)))
    blobs_de = torch.stack([fused.pack_blob(SPEC, {k: v.to(dev) for k, v in synthetic_params(a.seed + 100 + m).items()})
                            for m in mem_ids])

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    if a.bn_mode == "batch":
        from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
        from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops

        mcd_model = AlarconCNN1D(seed=a.seed, device=dev, params={k: v.to(dev) for k, v in synthetic_params(a.seed).items()})
        sync = torch.distributed.all_reduce if world > 1 else None

    def mcd_probs(i):
        if a.bn_mode == "running":
            return pinf.mcd_probs_local(blob_mcd, x_loc, a.passes, a.seed + i, start)
        # reference semantics: every pass normalises with the batch statistics of ALL windows
        return train_ops.forward_batch_stats(mcd_model, x_loc, a.passes, pass_base=i * a.passes, seed=a.seed,
                                             update_moving=True, sync=sync, window_offset=start, global_n=n_glob,
                                             max_samples=1 << 18)

    def step(i):
        ev[0].record()
        pm = mcd_probs(i)
        m_mcd = uq_ops.metrics(pm)
        s_mcd = pinf.aggregate_sums(m_mcd, y_loc)
        ev[1].record()
        if member_parallel:
            pd = pinf.de_probs_member_parallel(blobs_de, x_glob, world)
        else:
            pd = fused.fused_forward(x_loc, blobs_de, SPEC)[:, 0]
        m_de = uq_ops.metrics(pd)
        s_de = pinf.aggregate_sums(m_de, y_loc)
        sums = torch.stack([s_mcd, s_de])
        pdist.all_reduce_sum_(sums)
        ev[2].record()
        return sums

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    pdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mcd_ms = de_ms = 0.0
    for i in range(a.steps):
        sums = step(a.warmup + i)
        if a.steps <= 64:
            torch.cuda.synchronize()  # per-step split of the two phases (events)
            mcd_ms += ev[0].elapsed_time(ev[1])
            de_ms += ev[1].elapsed_time(ev[2])
    torch.cuda.synchronize()
    pdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.all_reduce_max(elapsed)
    agg_mcd = pinf.finalize_aggregates(sums[0])
    agg_de = pinf.finalize_aggregates(sums[1])

    ms = elapsed * 1e3 / a.steps
    value = n_glob * a.steps / elapsed
    macs = SPEC.forward_macs()
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "windows/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE is None else value / BASELINE,
            "dtype": "bf16",
            "data": "synthetic (random standardized 60x4 windows, random-init weights)",
            "config": {
                "model": "Alarcon 1D-CNN (6x[Conv1D-ReLU-BN-Dropout]+GAP+Dense, 853,441 params), input (60, 4)",
                "global_batch": n_glob,
                "seq_len": 60,
                "parallelism": f"dp{world}" + (f" (MCD: window-sharded; DE: member-parallel {a.members // world}/GPU + all_to_all)"
                                               if member_parallel else " (window-sharded, members replicated)"),
                "mcd_passes": a.passes,
                "de_members": a.members,
                "bn_mode_mcd": a.bn_mode,
                "windows_per_gpu_per_step": n_loc,
            },
            "extra": {
                "mcd_phase_ms": round(mcd_ms / max(a.steps, 1), 3),
                "de_phase_ms": round(de_ms / max(a.steps, 1), 3),
                "mcd_windows_per_s_per_gpu": round(n_loc / (mcd_ms / a.steps / 1e3), 1) if mcd_ms else None,
                "de_windows_per_s_per_gpu": round(n_loc / (de_ms / a.steps / 1e3), 1) if de_ms else None,
                "effective_tflops_per_gpu": round(n_loc * (a.passes + a.members) * 2 * macs / (ms / 1e3) / 1e12, 1),
                "mcd_mean_entropy": round(agg_mcd["mean_total_pred_entropy"], 6),
                "de_mean_mutual_info": round(agg_de["mean_mutual_info"], 6),
            },
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
