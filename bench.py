#!/usr/bin/env python3
"""Headline benchmark: 30s-windows/sec for MC Dropout T=50 & Deep Ensemble M=8 UQ inference.

Driver contract: ``python bench.py --gpus N --steps K --warmup W`` (self-launches N ranks, one per
GPU, when not already under torchrun) or ``torchrun --nproc-per-node N bench.py --gpus N ...``.
One *step* processes a fixed batch of ``--windows`` windows PER GPU (weak scaling) through the
complete UQ inference of both methods the reference evaluates
(``uncertainty_quantification/analyze_mcd_patient_level.py`` / ``analyze_de_patient_level.py``):

  1. MC Dropout, T=50 stochastic passes with the reference's semantics (``uq_techniques.py:22``,
     ``model(x, training=True)``): every pass normalises each BatchNorm with the batch statistics
     of the WHOLE window set (all ranks: SyncBN all-reduce per layer) and updates the moving
     averages; counter-based dropout masks keyed by the global window index; then the per-window
     mean / variance / entropy / expected entropy / MI reduction (HIP ``uq_reduce``);
  2. Deep Ensemble, M=8 members (inference BN, no dropout; ``uq_techniques.py:29``), member-parallel
     over the GPUs with an RCCL all_to_all of member probabilities over xGMI, then the same reduction;
  3. the 6 aggregate UQ scalars of each method, all-reduced over ranks.

Precision (``--precision``, default ``fp32``): the reference computes in fp32 (Keras defaults, no
mixed-precision policy), so the headline runs the fp32-faithful engine (``ops/x3.py``,
``csrc/x3_layers.hip``): every conv product is three fp16 MFMAs over a hi/lo split of both operands
with fp32 accumulation (22-bit operands, ~fp32 GEMM rounding), block 1 / BN / dropout / head in fp32.
``extra.fp32_deviation`` measures it against the fp32 PyTorch reference (``models/reference.py``) on a
fixed window subset.  The bf16 engine of rounds 1-2 is timed in the same run under ``extra.bf16``
(``--precision bf16`` makes it the headline, labelled ``dtype: bf16``).

``value`` = windows fully UQ-evaluated (both methods) per second over ALL GPUs.  Model: the
reference Alarcon 1D-CNN (853,441 params, 60 x 4 windows), random-init weights with non-trivial BN
statistics, synthetic standardised windows.  Timing: W untimed warmup steps, then K steps bracketed by
barrier + synchronize; the max over ranks is reported.  On the GPU a process group is formed even for
one rank (RCCL, world size 1), so the N=1 point runs the same code path as N=8.

``extra.train`` (``bench/train_extra.py``): BASELINE.json's training config (Adam, BCE, 1 x MI355X) on the
HIP training kernels -- the graphed single-model step at batch 1024 and 8192, 8 member-batched ensemble
members, and the loss deviation of 10 HIP steps from the same steps on fp32 autograd.

``--device cpu`` is a dry run of the same launcher / collectives / metrics on gloo with the fp32
reference model (CPU tests); its numbers are not performance claims.
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

METRIC = "30s-windows/sec for MCD T=50 & DE M=8 inference at 1/2/4/8 MI355X"
# The reference publishes no throughput number.  vs_baseline divides by OUR
# measurement of its exact loops in eager fp32 PyTorch on 1 x MI355X (bench/comparator.py, N=16384,
# MCD T=50 with BN batch statistics as the reference runs it + DE M=8 predict(batch 32) + NumPy UQ
# metrics): profiles/comparator_eager_fp32_batchbn_r1.json — the same MCD semantics as the headline
# (re-measured in round 3 on the current image: 4933.7, profiles/comparator_eager_fp32_batchbn_r3.json).
BASELINE = 4925.9
BASELINE_BASIS = ("eager fp32 PyTorch running the reference's loops (MCD: 50 x model(X, training=True) with BN batch "
                  "stats; DE: 8 x predict(batch 32)) on 1 x MI355X, profiles/comparator_eager_fp32_batchbn_r1.json")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); self-launched unless under torchrun")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--windows", type=int, default=16384, help="windows per GPU per step")
    ap.add_argument("--passes", type=int, default=50, help="MC Dropout passes T")
    ap.add_argument("--members", type=int, default=8, help="Deep Ensemble members M")
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                    help="headline engine: fp32-faithful (fp16x3 MFMA, the reference's precision; default) or bf16")
    ap.add_argument("--bn-mode", choices=["batch", "running"], default="batch",
                    help="MC-Dropout BatchNorm of the headline: per-pass batch statistics over the whole window set "
                         "(the reference's model(x, training=True); default) or running statistics (standard MC "
                         "Dropout)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the bf16 engine's timing (extra.bf16)")
    ap.add_argument("--no-deviation", action="store_true", help="skip the fp32 deviation block")
    ap.add_argument("--no-train", action="store_true", help="skip the training block (extra.train)")
    ap.add_argument("--deviation-windows", type=int, default=1024)
    ap.add_argument("--comm-steps", type=int, default=2,
                    help="steps after the timed region with every collective metered (extra.comm; 0: off)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = dry run of launcher + collectives on gloo with the fp32 reference model")
    return ap.parse_args(argv)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    # ---- launcher: spawn one worker per GPU BEFORE anything (incl. torch) touches the GPU
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import launch

    rc = launch.maybe_spawn(a.gpus, __file__, argv)
    if rc is not None:
        sys.exit(rc)
    if a.device == "cpu":
        os.environ.setdefault("APNEAUQ_DIST_BACKEND", "gloo")
        os.environ["CUDA_VISIBLE_DEVICES"] = ""
    else:
        os.environ.setdefault("APNEAUQ_FORCE_PG", "1")  # RCCL group even at world size 1 (same path as N=8)
    # the driver reads ONE JSON line from stdout: everything else any library prints there (RCCL's
    # version banner at communicator creation goes to fd 1 from C) is sent to stderr
    sys.stdout.flush()
    global _RESULT_FD
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)
    run(a)


_RESULT_FD = None


def _emit(line: str) -> None:
    sys.stdout.flush()
    if _RESULT_FD is None:
        print(line, flush=True)
    else:
        os.write(_RESULT_FD, (line + "\n").encode())


def run(a):
    import torch

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import uq as uq_ops
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import comm
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import dist as pdist
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import inference as pinf
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import launch

    cpu = a.device == "cpu"
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if cpu:
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(1, world_env)))
    launch.check_world(a.gpus, world_env, None if cpu else torch.cuda.device_count(), "cpu" if cpu else "cuda")
    info = pdist.init(device="cpu" if cpu else None)
    dev = info.device
    if not cpu and dev.type != "cuda":
        raise SystemExit("bench.py needs a GPU (use --device cpu for the dry run)")
    world, rank = info.world, info.rank
    n_loc = a.windows
    n_glob = n_loc * world

    # ---- resident data: the whole synthetic window set lives in HBM on every rank (fp32, as Keras feeds it)
    g = torch.Generator(device="cpu").manual_seed(a.seed)
    x32_glob = torch.randn(n_glob, 60, 4, generator=g)
    y_glob = (torch.rand(n_glob, generator=g) < 0.3).to(torch.int32)
    x_glob = x32_glob.to(dev)
    y_glob = y_glob.to(dev)
    start, stop = pdist.shard_range(n_glob, rank, world)
    x_loc = x_glob[start:stop].contiguous()
    y_loc = y_glob[start:stop].contiguous()

    params_mcd = {k: v.to(dev) for k, v in R.synthetic_params(SPEC, a.seed).items()}
    member_parallel = world > 1 and a.members % world == 0
    mem_ids = (list(range(rank * (a.members // world), (rank + 1) * (a.members // world)))
               if member_parallel else list(range(a.members)))
    params_de = [{k: v.to(dev) for k, v in R.synthetic_params(SPEC, a.seed + 100 + m).items()} for m in mem_ids]
    use_pg = torch.distributed.is_available() and torch.distributed.is_initialized()
    # SyncBN all-reduce of the fp64 BN moment sums (one per BN layer and pass chunk)
    sync = ((lambda t: comm.run("syncbn_all_reduce", t, lambda: torch.distributed.all_reduce(t)))
            if (use_pg and not cpu) or world > 1 else None)

    def make(precision):
        if cpu:
            return _CpuEngine(R, SPEC, params_mcd, params_de, world, start, n_glob, a.seed, a.passes)
        cls = _X3Engine if precision == "fp32" else _Bf16Engine
        return cls(R, SPEC, params_mcd, params_de, world, start, n_glob, a.seed, a.passes, sync)

    def timed(engine, mode: str, steps: int, warmup: int, step_base: int, comm_steps: int = 0):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if not cpu else None
        phase = [0.0, 0.0]

        def step(i, meter=None):
            if ev:
                ev[0].record()
            t0 = time.perf_counter()
            if meter is not None:
                meter.step()
                meter.phase("mcd")
            pm = engine.mcd(mode, x_loc, step_base + i)
            s_mcd = pinf.aggregate_sums(uq_ops.metrics(pm), y_loc)
            if ev:
                ev[1].record()
            t1 = time.perf_counter()
            if meter is not None:
                meter.phase("de")
            if member_parallel:
                pd = pinf.all_to_all_members(engine.de(x_glob), world)
            else:
                pd = engine.de(x_loc)
            s_de = pinf.aggregate_sums(uq_ops.metrics(pd), y_loc)
            sums = torch.stack([s_mcd, s_de])
            if meter is not None:
                meter.phase("aggregate")
            pdist.all_reduce_sum_(sums)
            if ev:
                ev[2].record()
            return sums, (t0, t1, time.perf_counter())

        for i in range(warmup):
            step(i)
        if not cpu:
            torch.cuda.synchronize()
        pdist.barrier()
        if not cpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        sums = None
        for i in range(steps):
            sums, tt = step(warmup + i)
            if ev and steps <= 64:
                torch.cuda.synchronize()  # per-step split of the two phases (events)
                phase[0] += ev[0].elapsed_time(ev[1])
                phase[1] += ev[1].elapsed_time(ev[2])
            elif cpu:
                phase[0] += (tt[1] - tt[0]) * 1e3
                phase[1] += (tt[2] - tt[1]) * 1e3
        if not cpu:
            torch.cuda.synchronize()
        pdist.barrier()
        if not cpu:
            torch.cuda.synchronize()
        elapsed = pdist.all_reduce_max(time.perf_counter() - t0)
        # collective accounting (extra.comm): a few MORE steps after the timed region, metered (events
        # around every collective), so the timed steps carry no instrumentation
        comm_rec = None
        if comm_steps > 0:
            meter = comm.CommMeter()
            with comm.metering(meter):
                for i in range(comm_steps):
                    step(warmup + steps + i, meter)
            comm_rec = meter.summary()
            comm_rec["note"] = "per step; metered on steps after the timed region; ms = HIP-event time on the compute stream"
            pdist.barrier()
        return elapsed, sums, phase, comm_rec

    head_prec = "fp32" if cpu else a.precision
    engine = make(head_prec)
    elapsed, sums, phase, comm_rec = timed(engine, a.bn_mode, a.steps, a.warmup, 0, comm_steps=a.comm_steps)
    agg_mcd = pinf.finalize_aggregates(sums[0])
    agg_de = pinf.finalize_aggregates(sums[1])
    ms = elapsed * 1e3 / a.steps
    value = n_glob * a.steps / elapsed

    deviation = None
    if not cpu and not a.no_deviation:
        deviation = engine.deviation(x_glob[: a.deviation_windows], y_glob[: a.deviation_windows])

    secondary = None
    if not cpu and not a.no_secondary:
        other = "bf16" if head_prec == "fp32" else "fp32"
        del engine
        torch.cuda.empty_cache()
        eng2 = make(other)
        k2 = max(1, min(a.steps, 10))
        e2, s2, ph2, _ = timed(eng2, a.bn_mode, k2, 1, 10_000)
        secondary = {
            "precision": other,
            "value": round(n_glob * k2 / e2, 1),
            "ms_per_step": round(e2 * 1e3 / k2, 3),
            "steps": k2,
            "mcd_phase_ms": round(ph2[0] / k2, 3),
            "de_phase_ms": round(ph2[1] / k2, 3),
            "mcd_mean_entropy": round(pinf.finalize_aggregates(s2[0])["mean_total_pred_entropy"], 6),
        }
        if not a.no_deviation:
            secondary["fp32_deviation"] = eng2.deviation(x_glob[: a.deviation_windows], y_glob[: a.deviation_windows])

    train = None
    if not cpu and not a.no_train:  # BASELINE.json config #2: the training step (every rank trains its own models)
        from bench import train_extra

        torch.cuda.empty_cache()
        train = train_extra.measure(dev, a.seed)

    fp32_paths = None
    if not cpu and not a.no_train:  # the reference-precision paths of the other architectures + fp32 training
        # single-device numbers: rank 0 alone, between barriers (the other ranks wait), distributed=False
        from bench import fp32_micro

        pdist.barrier()
        if rank == 0:
            torch.cuda.empty_cache()
            fp32_paths = fp32_micro.measure(reps=2, steps=20, precisions=("fp32",))
            fp32_paths["note"] = ("pooled ensemble_cnn members (MaxPool1D after blocks 1-5) at precision fp32: DE / "
                                  "running-BN MCD on the fused fp16x3 kernel, batch-BN MCD layer-wise; fp32 training "
                                  "steps (train_precision='fp32') of the reference and pooled CNN; best of 2; "
                                  "measured on rank 0 alone (single device, no collectives)")
        pdist.barrier()

    macs = SPEC.forward_macs()
    devices = pdist.gather_device_ids()  # collective: every rank
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
            "vs_baseline": None if (BASELINE is None or cpu or head_prec != "fp32") else round(value / BASELINE, 3),
            "vs_baseline_basis": BASELINE_BASIS if a.bn_mode == "batch" else
            BASELINE_BASIS + " (NOTE: headline run in bn_mode=running; semantics differ)",
            "dtype": "fp32" if head_prec == "fp32" else "bf16",
            "compute": ("fp32-faithful: conv products as 3 fp16 MFMAs over hi/lo splits of both operands, fp32 "
                        "accumulate; block 1, BN (fp64 moments), dropout, GAP, Dense, sigmoid in fp32") if head_prec == "fp32"
            else "bf16 MFMA operands, fp32 accumulate",
            "data": "synthetic (random standardized 60x4 windows, random-init weights)",
            "config": {
                "model": "Alarcon 1D-CNN (6x[Conv1D-ReLU-BN-Dropout]+GAP+Dense, 853,441 params), input (60, 4)",
                "global_batch": n_glob,
                "seq_len": 60,
                "parallelism": f"dp{world}" + (f" (MCD: window-sharded + SyncBN; DE: member-parallel {a.members // world}/GPU"
                                               " + all_to_all)" if member_parallel else
                                               (" (MCD: window-sharded + SyncBN; DE: members replicated)" if world > 1 else "")),
                "mcd_passes": a.passes,
                "de_members": a.members,
                "bn_mode_mcd": a.bn_mode,
                "windows_per_gpu_per_step": n_loc,
            },
            "backend": info.backend,
            "devices": devices,
            "extra": {
                "mcd_phase_ms": round(phase[0] / max(a.steps, 1), 3),
                "de_phase_ms": round(phase[1] / max(a.steps, 1), 3),
                "mcd_windows_per_s_per_gpu": round(n_loc / (phase[0] / a.steps / 1e3), 1) if phase[0] else None,
                "de_windows_per_s_per_gpu": round(n_loc / (phase[1] / a.steps / 1e3), 1) if phase[1] else None,
                "effective_tflops_per_gpu": round(n_loc * (a.passes + a.members) * 2 * macs / (ms / 1e3) / 1e12, 1),
                "mcd_mean_entropy": round(agg_mcd["mean_total_pred_entropy"], 6),
                "de_mean_mutual_info": round(agg_de["mean_mutual_info"], 6),
                "comm": comm_rec,
                "fp32_deviation": deviation,
                ("bf16" if head_prec == "fp32" else "fp32"): secondary,
                "train": train,
                "fp32_paths": fp32_paths,
            },
        }
        _emit(json.dumps(out))
    pdist.shutdown()


def _mcd_deviation(R, spec, params, x32, y, T, seed, base, run_hip, uq_ops, pinf):
    """max / mean |dp| and aggregate deltas of one engine's batch-BN and running-BN MC Dropout against
    the fp32 reference forward on the same weights, masks and inputs."""
    import torch

    n = x32.shape[0]
    ids = torch.arange(n, device=x32.device)
    agg = {}
    for mode in ("batch", "running"):
        ph = run_hip(mode)
        pr = torch.stack([R.forward(spec, params, x32, dropout=True, bn_batch_stats=(mode == "batch"), seed=seed,
                                    pass_id=base + t, sample_ids=ids).reshape(-1) for t in range(T)])
        ah = pinf.finalize_aggregates(pinf.aggregate_sums(uq_ops.metrics(ph), y))
        ar = pinf.finalize_aggregates(pinf.aggregate_sums(uq_ops.metrics_eager(pr), y))
        agg[mode] = {
            "max_abs_dp": float((ph - pr).abs().max()),
            "mean_abs_dp": float((ph - pr).abs().mean()),
            "aggregates_hip": {k: round(v, 6) for k, v in ah.items()},
            "aggregates_delta": {k: float(f"{ah[k] - ar[k]:.3e}") for k in ah},
        }
    return agg


class _X3Engine:
    """fp32-faithful engine (ops/x3.py): batch-BN MCD and DE on the fp16x3 layer kernels."""

    def __init__(self, R, spec, params_mcd, params_de, world, start, n_glob, seed, passes, sync):
        from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import x3

        self.x3, self.R, self.spec = x3, R, spec
        self.world, self.start, self.n_glob, self.seed, self.passes, self.sync = world, start, n_glob, seed, passes, sync
        self.params_mcd, self.params_de = params_mcd, params_de
        # the MCD model owns its own parameter copy: its moving statistics are mutated every pass
        self.m_mcd = x3.X3Model(spec, [{k: v.clone() for k, v in params_mcd.items()}])
        self.m_de = x3.X3Model(spec, params_de)

    def mcd(self, mode, x_loc, i):
        if mode == "running":
            return self.x3.forward_running(self.m_mcd, x_loc, n_pass=self.passes, dropout=True, seed=self.seed,
                                           pass_offset=i * self.passes, window_offset=self.start)[0]
        return self.x3.mcd_batch(self.m_mcd, x_loc, self.passes, seed=self.seed, pass_base=i * self.passes,
                                 window_offset=self.start, update_moving=True, sync=self.sync, global_n=self.n_glob)

    def de(self, x):
        return self.x3.forward_running(self.m_de, x)[:, 0]

    def deviation(self, x32, y):
        import torch

        from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import uq as uq_ops
        from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import inference as pinf

        x3, R, spec = self.x3, self.R, self.spec
        out = {"windows": x32.shape[0], "engine": "fp32-faithful (fp16x3)",
               "reference": "models/reference.py forward in fp32 (same weights, masks, fp32 input)"}
        with torch.no_grad():
            de = x3.X3Model(spec, self.params_de[:1])
            p_hip = x3.forward_running(de, x32)[0, 0]
            p_ref = R.forward(spec, self.params_de[0], x32, training=False).reshape(-1)
            out["de_member_max_abs_dp"] = float((p_hip - p_ref).abs().max())
            T, seed, base = self.passes, self.seed + 555, 777
            mm = x3.X3Model(spec, [{k: v.clone() for k, v in self.params_mcd.items()}])

            def run_hip(mode):
                if mode == "batch":
                    return x3.mcd_batch(mm, x32, T, seed=seed, pass_base=base, update_moving=False)
                return x3.forward_running(mm, x32, n_pass=T, dropout=True, seed=seed, pass_offset=base)[0]

            agg = _mcd_deviation(R, spec, self.params_mcd, x32, y, T, seed, base, run_hip, uq_ops, pinf)
            out["mcd_T"] = T
            out["mcd_batch_bn"] = agg["batch"]
            out["mcd_running_bn"] = agg["running"]
        return out


class _Bf16Engine:
    """bf16 HIP kernels of rounds 1-2: batch-BN MCD on the layer-wise kernels, running-BN MCD and DE fused."""

    def __init__(self, R, spec, params_mcd, params_de, world, start, n_glob, seed, passes, sync):
        import torch

        from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
        from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused

        self.R, self.spec, self.fused = R, spec, fused
        self.world, self.start, self.n_glob, self.seed, self.passes, self.sync = world, start, n_glob, seed, passes, sync
        self.params_mcd = params_mcd
        self.params_de = params_de
        # batch-BN MCD: samples (passes x windows) per layer-kernel launch, all T passes in one chunk when
        # the bf16 activations fit in half of the free HBM (halved until they do)
        env = os.environ.get("APNEAUQ_MCD_MAX_SAMPLES")
        dev = params_mcd["conv1d_1/kernel"].device
        if env:
            self.max_samples = int(env)
        else:
            free = torch.cuda.mem_get_info(dev)[0]
            per_sample = 64 * sum(b.filters for b in spec.blocks[1:]) * 2
            ms = 1 << 20
            while ms > (1 << 16) and ms * per_sample > 0.5 * free:
                ms >>= 1
            if world > 1:  # every rank must chunk the passes identically (one SyncBN all-reduce per chunk)
                import torch.distributed as dist

                t = torch.tensor([ms], dtype=torch.int64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MIN)
                ms = int(t.item())
            self.max_samples = ms
        self.blob_mcd = fused.pack_blob(spec, params_mcd).unsqueeze(0)
        self.blobs_de = torch.stack([fused.pack_blob(spec, p) for p in params_de])
        self.model = AlarconCNN1D(seed=seed, device=dev, params={k: v.clone() for k, v in params_mcd.items()})

    def mcd(self, mode, x_loc, i):
        import torch

        from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops
        from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import inference as pinf

        xb = x_loc.to(torch.bfloat16)
        if mode == "running":
            return pinf.mcd_probs_local(self.blob_mcd, xb, self.passes, self.seed + i, self.start)
        return train_ops.forward_batch_stats(self.model, xb, self.passes, pass_base=i * self.passes, seed=self.seed,
                                             update_moving=True, sync=self.sync, window_offset=self.start,
                                             global_n=self.n_glob, max_samples=self.max_samples)

    def de(self, x):
        import torch

        return self.fused.fused_forward(x.to(torch.bfloat16), self.blobs_de, self.spec)[:, 0]

    def deviation(self, x32, y):
        import torch

        from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
        from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops, uq as uq_ops
        from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import inference as pinf

        R, spec = self.R, self.spec
        xb = x32.to(torch.bfloat16)
        out = {"windows": x32.shape[0], "engine": "bf16",
               "reference": "models/reference.py forward in fp32 (same weights, masks, fp32 input)"}
        with torch.no_grad():
            p_hip = self.fused.fused_forward(xb, self.blobs_de[:1], spec)[0, 0]
            p_ref = R.forward(spec, self.params_de[0], x32, training=False).reshape(-1)
            out["de_member_max_abs_dp"] = float((p_hip - p_ref).abs().max())
            T, seed, base = self.passes, self.seed + 555, 777

            def run_hip(mode):
                if mode == "batch":
                    model = AlarconCNN1D(seed=seed, device=x32.device,
                                         params={k: v.clone() for k, v in self.params_mcd.items()})
                    return train_ops.forward_batch_stats(model, xb, T, pass_base=base, seed=seed, update_moving=False)
                return self.fused.fused_forward(xb, self.blob_mcd, spec, n_pass=T, dropout=True, seed=seed,
                                                pass_offset=base)[0]

            agg = _mcd_deviation(R, spec, self.params_mcd, x32, y, T, seed, base, run_hip, uq_ops, pinf)
            out["mcd_T"] = T
            out["mcd_batch_bn"] = agg["batch"]
            out["mcd_running_bn"] = agg["running"]
        return out


class _CpuEngine:
    """fp32 reference model on the CPU (dry run of the distributed bench on gloo)."""

    def __init__(self, R, spec, params_mcd, params_de, world, start, n_glob, seed, passes):
        self.R, self.spec, self.world, self.start, self.n_glob = R, spec, world, start, n_glob
        self.seed, self.passes = seed, passes
        self.params_mcd, self.params_de = params_mcd, params_de

    def _sync_hook(self, h):
        import torch
        import torch.distributed as dist

        s = torch.stack([h.sum(dim=(0, 1)), (h * h).sum(dim=(0, 1))]).double()
        cnt = torch.tensor([float(h.shape[0] * h.shape[1])], dtype=torch.float64)
        if dist.is_initialized() and self.world > 1:
            from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import comm

            comm.run("syncbn_all_reduce", s, lambda: dist.all_reduce(s))
            comm.run("syncbn_all_reduce", cnt, lambda: dist.all_reduce(cnt))
        mean = s[0] / cnt
        var = (s[1] / cnt - mean * mean).clamp_min(0)
        return mean.float(), var.float()

    def mcd(self, mode, x_loc, i):
        import torch

        ids = torch.arange(self.start, self.start + x_loc.shape[0])
        with torch.no_grad():
            return torch.stack([self.R.forward(self.spec, self.params_mcd, x_loc, dropout=True,
                                               bn_batch_stats=(mode == "batch"), seed=self.seed,
                                               pass_id=i * self.passes + t, sample_ids=ids,
                                               bn_stats_hook=self._sync_hook if mode == "batch" else None).reshape(-1)
                                for t in range(self.passes)])

    def de(self, x):
        import torch

        with torch.no_grad():
            return torch.stack([self.R.forward(self.spec, p, x, training=False).reshape(-1) for p in self.params_de])


if __name__ == "__main__":
    main()
