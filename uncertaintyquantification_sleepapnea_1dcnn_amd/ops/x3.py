"""Host side of the fp32-faithful layer-wise inference engine (``csrc/x3_layers.hip``).

The reference computes in fp32 (Keras defaults; no mixed-precision policy anywhere in
``/root/reference``).  This engine reproduces its inference workloads at that precision on the MI355X
matrix cores: every Conv1D operand is split into two fp16 halves (``v = hi + lo``, 22 significant
bits) and each product is formed by three ``v_mfma_f32_16x16x32_f16`` (hi*hi + hi*lo + lo*hi) with
fp32 accumulation; block 1 (Cin = 4) runs in plain fp32 FMAs; BatchNorm moments are fp64 across
tiles; BN apply, dropout, GAP, Dense and sigmoid are fp32.  Workloads:

* :func:`mcd_batch` -- MC Dropout exactly as the reference runs it (``uq_techniques.py:22``,
  ``model(x, training=True)`` T times on the whole test set): per-pass batch statistics of every BN
  over all windows (SyncBN over ranks), dropout, the moving-average side effect;
* :func:`forward_running` -- BN on moving statistics: Deep-Ensemble ``predict`` of M members
  (``uq_techniques.py:29``) or standard MC Dropout (dropout on).

Weights are packed once per model set (:class:`X3Model`); activations live in HBM between the six
layer launches (fp32 ReLU outputs; the dropout mask of block l is drawn from the counter hash by the
block that stages it, block l + 1).
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional, Sequence

import torch

from ..models.spec import ModelSpec
from . import _ext, fused, rng

CH = fused.FUSED_CHANNELS
KS = fused.FUSED_KSIZES
STAT_SLOTS = 16  # csrc/x3_args.h kStatSlots
TILE = 4         # samples per layer-kernel tile
CK = 32          # input channels per staged chunk
# bytes of activation workspace per sample: ping-pong fp32 buffers of 192 + 256 channels x 60 steps
# (+ the block-1 output: per window for batch-BN MC Dropout, per window and member for the Deep Ensemble;
# budgeted per sample, the conservative bound)
BYTES_PER_SAMPLE = 60 * (192 + 256) * 4
R1_BYTES = 60 * 128 * 4


def supports(spec: ModelSpec) -> bool:
    return fused.supports(spec)


def pack_conv(kernel: torch.Tensor):
    """Keras conv kernel (k, Cin, Cout) fp32 -> (fp16 hi/lo MFMA fragments, 2^-sw).

    The kernel is pre-scaled by an exact power of two ``2^sw`` (largest |w| -> [2^13, 2^14)) so that
    hi = fp16(w) and lo = fp16(w - hi) are both normal; the layer kernel multiplies its fp32 accumulator
    by ``2^-sw``.  Fragment layout ``[chunk][tap][ct][hi|lo][lane][8]``: lane l of the A fragment of output
    tile ct holds ``W[tap][32 chunk + 8 (l >> 4) + e][16 ct + (l & 15)]``, e = 0..7 (v_mfma_f32_16x16x32_f16
    A-operand map: row = l & 15, k = 8 (l >> 4) + e)."""
    k, cin, cout = kernel.shape
    assert cin % CK == 0 and cout % 16 == 0
    w = kernel.detach().to(torch.float64)
    amax = float(w.abs().max()) if w.numel() else 0.0
    sw = 13 - math.frexp(amax)[1] + 1 if amax > 0 else 0  # amax * 2^sw in [2^13, 2^14)
    ws = (w * (2.0 ** sw)).float()
    hi = ws.half()
    lo = (ws - hi.float()).half()
    nch, nct = cin // CK, cout // 16

    def frag(p):  # (k, cin, cout) -> (nch, k, nct, 64, 8)
        v = p.reshape(k, nch, 4, 8, nct, 16)            # tap, chunk, h, e, ct, m
        return v.permute(1, 0, 4, 2, 5, 3).reshape(nch, k, nct, 64, 8)

    fr = torch.stack([frag(hi), frag(lo)], dim=3)        # (nch, k, nct, 2, 64, 8)
    return fr.contiguous().reshape(-1), 2.0 ** (-sw)


def unpack_conv(fr: torch.Tensor, wscale: float, k: int, cin: int, cout: int) -> torch.Tensor:
    """Inverse of :func:`pack_conv`: the fp32 kernel hi + lo (times 2^-sw), (k, Cin, Cout)."""
    nch, nct = cin // CK, cout // 16
    v = fr.reshape(nch, k, nct, 2, 4, 16, 8).float()
    w = v[:, :, :, 0] + v[:, :, :, 1]                      # (nch, k, nct, h, m, e)
    w = w.permute(1, 0, 3, 5, 2, 4).reshape(k, cin, cout)  # tap, chunk, h, e, ct, m
    return w.double().mul(wscale).float()


class X3Model:
    """Packed parameters of G models (ensemble members) for the layer kernels.

    ``params``: list of Keras-named parameter dicts (``models/reference.py``).  With one model the BN
    moving statistics are views of the caller's tensors when they are contiguous fp32 on the device
    (the batch-statistics MC Dropout updates them in place, as ``model(x, training=True)`` does)."""

    def __init__(self, spec: ModelSpec, params: Sequence[Dict[str, torch.Tensor]], device=None):
        if not supports(spec):
            raise ValueError("the x3 engine implements the reference (60, 4) no-pool architecture")
        self.spec = spec
        self.G = len(params)
        dev = torch.device(device) if device is not None else params[0]["conv1d_1/kernel"].device
        if dev.type == "cuda" and dev.index is None:  # "cuda" == the current device ("cuda" != "cuda:0")
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        f32 = dict(dtype=torch.float32, device=dev)
        self.w1 = torch.stack([p["conv1d_1/kernel"].to(**f32) for p in params]).contiguous()  # (G, 7, 4, 128)
        self.b1 = torch.stack([p["conv1d_1/bias"].to(**f32) for p in params]).contiguous()
        self.wfrag: List[Optional[torch.Tensor]] = [None]
        self.wscale: List[Optional[torch.Tensor]] = [None]
        self.bias: List[torch.Tensor] = [self.b1]
        for l in range(1, 6):
            frs, scs = [], []
            for p in params:
                fr, sc = pack_conv(p[f"conv1d_{l + 1}/kernel"].to(dev))
                frs.append(fr)
                scs.append(sc)
            self.wfrag.append(torch.stack(frs).contiguous())
            self.wscale.append(torch.tensor(scs, **f32))
            self.bias.append(torch.stack([p[f"conv1d_{l + 1}/bias"].to(**f32) for p in params]).contiguous())
        self.bn = []
        for l in range(6):
            names = [f"batchnorm_{l + 1}/{n}" for n in ("gamma", "beta", "moving_mean", "moving_variance")]
            entry = []
            for n in names:
                src = params[0][n]
                if self.G == 1 and src.device == dev and src.dtype == torch.float32 and src.is_contiguous():
                    entry.append(src.view(1, -1))  # in-place moving updates reach the caller's model
                else:
                    entry.append(torch.stack([p[n].to(**f32) for p in params]).contiguous())
            self.bn.append(entry)
        self.dw = torch.stack([p["output_layer/kernel"].to(**f32).reshape(-1) for p in params]).contiguous()
        self.db = torch.stack([p["output_layer/bias"].to(**f32).reshape(-1) for p in params]).reshape(-1).contiguous()
        self._ws: Dict[tuple, "_Workspace"] = {}

    def workspace(self, samples: int, n_r1: int, groups: int) -> "_Workspace":
        """One workspace at a time (the buffers are large), kept while it is big enough: a call with
        fewer samples / windows / groups (a tail batch) reuses it instead of reallocating."""
        ws = self._ws.get("ws")
        if ws is None or ws.samples < samples or ws.n_r1 < n_r1 or ws.groups < groups:
            self._ws.clear()
            ws = self._ws["ws"] = _Workspace(self.device, samples, n_r1, groups)
        return ws


class _Workspace:
    def __init__(self, dev, samples: int, n_r1: int, groups: int):
        self.samples, self.n_r1, self.groups = int(samples), int(n_r1), max(int(groups), 1)
        f32 = dict(dtype=torch.float32, device=dev)
        self.r1 = torch.empty(n_r1 * 60 * CH[1], **f32)
        self.buf = [torch.empty(samples * 60 * 192, **f32), torch.empty(samples * 60 * 256, **f32)]
        self.sums = torch.empty(samples * 2 * CH[6], **f32)
        self.out = torch.empty(samples, **f32)
        self.stats = [torch.zeros(max(groups, 1) * STAT_SLOTS * 2 * CH[l + 1], dtype=torch.float64, device=dev)
                      for l in range(6)]
        self.aff = [torch.empty(max(groups, 1) * 2 * CH[l + 1], **f32) for l in range(6)]
        # range-safe fp16 split of block l+2's input (csrc/x3_layers.hip sample_prescale).  Moving statistics:
        # the max of R_l per sample (fp32 bits; block 1: per window and member) and the channel maxima of
        # each affine.  Batch moments: one power of two per group, from the moments themselves, folded into
        # the affine (x3_aff gscale).  Cost: profiles/x3_mask_side_r4.md.
        self.smax = [torch.zeros(n_r1 if l == 0 else samples, dtype=torch.int32, device=dev) for l in range(5)]
        self.amax = [torch.zeros(max(groups, 1) * 2, **f32) for l in range(6)]
        self.gscale = [torch.ones(max(groups, 1), **f32) for l in range(5)] + [None]

    def smax_out(self, l: int, k: int) -> Optional[torch.Tensor]:
        """Block l+1's per-sample maxima (first k samples, zeroed: atomicMax targets); None for block 6."""
        if l >= 5:
            return None
        return self.smax[l][:k].zero_()


def _ops():
    return _ext.ops()


# layers (x3_layer index 1..4 = blocks 2..5) whose epilogue draws its block's dropout mask and stores it in
# the output's sign bit; the others store plain ReLU output and their consumer draws the mask while it
# stages the input (which side has the slack differs per layer: profiles/x3_mask_side_r4.md).
# APNEAUQ_X3_SIGN_MASK="2,3" overrides (A/B probes).
_SIGN_DEFAULT = "2,4"


def _sign_layers() -> frozenset:
    v = os.environ.get("APNEAUQ_X3_SIGN_MASK", _SIGN_DEFAULT)
    return frozenset(int(t) for t in v.replace(" ", "").split(",") if t)


def _sign(l: int, sl: frozenset):
    """(sign_in, sign_out) of x3_layer l."""
    return (l - 1) in sl and l >= 2, l in sl and l <= 4


def _dsc(rate: float) -> float:
    return 1.0 / (1.0 - rate) if rate < 1.0 else 0.0


def _sync_stats(sync: Callable, st: torch.Tensor, groups: int, c: int) -> None:
    """SyncBN: add the interleaved slots locally, all-reduce one slot's worth (groups x 2 x C fp64) and
    leave the global sums in slot 0 (the aff kernel adds all slots)."""
    v = st[: groups * STAT_SLOTS * 2 * c].view(groups, STAT_SLOTS, 2 * c)
    tot = v.sum(1)
    sync(tot)
    v.zero_()
    v[:, 0].copy_(tot)


def _max_samples(dev, per_sample: int, frac: float = 0.45) -> int:
    """Samples (windows x passes / members) per layer launch: at most ``frac`` of the free HBM and at most
    ``APNEAUQ_X3_WS_GB`` (default 20 GB) of activation workspace, so that the engine co-resides with
    other work (one 50-pass chunk of 16384 windows would hold ~88 GB).  Batch-BN MC Dropout over 16384
    windows, T = 50: 219.2-220.3 ms in one chunk (100 GB cap), 219.6-220.0 ms in 12-GB chunks
    (``profiles/x3_epilogue_ab_r3.md``): pass chunks of >= 30 k samples keep the launches full."""
    import os

    free = torch.cuda.mem_get_info(dev)[0]
    cap = float(os.environ.get("APNEAUQ_X3_WS_GB", "20")) * 2 ** 30
    return max(1, int(min(free * frac, cap)) // per_sample)


@torch.no_grad()
def mcd_batch(model: X3Model, x: torch.Tensor, n_pass: int, seed: int, pass_base: int = 0, window_offset: int = 0,
              update_moving: bool = True, sync: Optional[Callable] = None, global_n: Optional[int] = None,
              max_samples: Optional[int] = None, grid: int = 0) -> torch.Tensor:
    """MC Dropout with BN on per-pass batch statistics (reference semantics), fp32-faithful: (T, N).

    ``x``: (N, 60, 4) windows of this rank; with ``sync`` (all-reduce of fp64 tensors) the BN moments are
    those of all ``global_n`` windows of all ranks.  Passes are processed in chunks that fit the device
    (statistics are per pass, so chunking is exact; every rank must use the same chunking).  ``grid``:
    persistent workgroups per layer launch (0: one per CU)."""
    assert model.G == 1, "mcd_batch runs one model"
    spec, o = model.spec, _ops()
    x = x.to(device=model.device, dtype=torch.float32).contiguous()
    n = x.shape[0]
    gn = int(global_n or n)
    if max_samples is None:
        max_samples = _max_samples(model.device, BYTES_PER_SAMPLE + R1_BYTES)
        if sync is not None:  # identical chunking on every rank
            t = torch.tensor([float(max_samples)], dtype=torch.float64, device=model.device)
            import torch.distributed as dist

            from ..parallel import comm

            comm.run("chunking_all_reduce_min", t, lambda: dist.all_reduce(t, op=dist.ReduceOp.MIN))
            max_samples = int(t.item())
    ref_n = n
    if sync is not None and global_n:
        import torch.distributed as dist

        w = dist.get_world_size() if dist.is_initialized() else 1
        ref_n = -(-gn // w)
    if ref_n > max_samples:  # one pass of all windows does not fit: window-chunked two-phase schedule
        return _mcd_batch_windowed(model, x, n_pass, seed, pass_base, window_offset, update_moving, sync, gn,
                                   max_samples)
    cap = max(1, min(n_pass, max_samples // max(ref_n, 1)))
    n_chunks = -(-n_pass // cap)
    chunk = -(-n_pass // n_chunks)
    ws = model.workspace(chunk * n, n, chunk)
    inv_count = 1.0 / (gn * 60.0)
    thr = [rng.dropout_threshold(b.dropout) for b in spec.blocks]
    dsc = [_dsc(b.dropout) for b in spec.blocks]
    eps, mom = float(spec.bn_epsilon), float(spec.bn_momentum)
    seed = int(seed) & ((1 << 63) - 1)
    sl = _sign_layers()
    out = torch.empty(n_pass, n, dtype=torch.float32, device=model.device)
    # block 1 once: no dropout precedes it, so every pass sees the same R_1 and the same moments
    ws.stats[0].zero_()
    o.x3_l1(x, model.w1, model.b1, ws.r1, ws.stats[0], n, 1, None)
    if sync is not None:
        _sync_stats(sync, ws.stats[0], 1, CH[1])
    g, b, mm, mv = model.bn[0]
    o.x3_aff(ws.stats[0], g, b, mm, mv, ws.aff[0], CH[1], 1, 0, bool(update_moving), n_pass, inv_count, eps, mom, dsc[0],
             None, ws.gscale[0])
    for t0 in range(0, n_pass, chunk):
        tc = min(chunk, n_pass - t0)
        pb = int(pass_base) + t0
        for l in range(1, 6):
            c = CH[l + 1]
            st = ws.stats[l]
            st[: tc * STAT_SLOTS * 2 * c].zero_()
            src = ws.r1 if l == 1 else ws.buf[(l - 2) % 2]
            dst = ws.sums if l == 5 else ws.buf[(l - 1) % 2]
            o.x3_layer(l, src, dst, model.wfrag[l], 0, model.bias[l], model.wscale[l], 0, ws.aff[l - 1],
                       0 if l == 1 else 2 * CH[l], st, n, tc, l == 1, thr[l - 1], thr[l], seed, pb,
                       int(window_offset), int(grid), None, None, None, ws.gscale[l - 1], *_sign(l, sl))
            if sync is not None:
                _sync_stats(sync, st, tc, c)
            g, b, mm, mv = model.bn[l]
            o.x3_aff(st, g, b, mm, mv, ws.aff[l], c, tc, 0, bool(update_moving), 1, inv_count, eps, mom, dsc[l],
                     None, ws.gscale[l])
        o.x3_head(ws.sums, ws.aff[5], 2 * CH[6], model.dw, model.db, 0, ws.out, n, tc, False)
        out[t0: t0 + tc].copy_(ws.out[: tc * n].view(tc, n))
    return out


def _mcd_batch_windowed(model: X3Model, x: torch.Tensor, n_pass: int, seed: int, pass_base: int,
                        window_offset: int, update_moving: bool, sync: Optional[Callable], gn: int,
                        max_samples: int) -> torch.Tensor:
    """Batch-BN MC Dropout when even one pass over the rank's windows exceeds the activation budget.

    The BN moments of block l are moments over ALL windows, and block l+1 cannot start before they are
    known, so with window chunks the activations below block l are recomputed: for l = 1..6 every chunk
    runs blocks 1..l with the (already final) affines of blocks 1..l-1 and accumulates block l's moments;
    a last sweep runs the whole network with all affines and the head.  The dropout masks are counters of
    (seed, block, pass, global window id), so the recomputed activations are the same numbers, and the
    result equals the one-shot schedule up to the order of the fp64 moment sums.  Cost: 21 block
    evaluations per pass instead of 6 (only beyond ~2 M windows per 288-GB GPU)."""
    spec, o = model.spec, _ops()
    n = x.shape[0]
    wc = max(1, int(max_samples))
    bounds = [(s, min(n, s + wc)) for s in range(0, n, wc)]
    ws = model.workspace(wc, wc, 1)
    inv_count = 1.0 / (gn * 60.0)
    thr = [rng.dropout_threshold(b.dropout) for b in spec.blocks]
    dsc = [_dsc(b.dropout) for b in spec.blocks]
    eps, mom = float(spec.bn_epsilon), float(spec.bn_momentum)
    seed = int(seed) & ((1 << 63) - 1)
    sl = _sign_layers()
    out = torch.empty(n_pass, n, dtype=torch.float32, device=model.device)

    def run(s: int, e: int, upto: int, pb: int, stats_layer: int) -> None:
        """Blocks 1..upto+1 over windows [s, e) of pass pb; moments of block stats_layer+1 into its slots."""
        m = e - s
        o.x3_l1(x[s:e], model.w1, model.b1, ws.r1, ws.stats[0] if stats_layer == 0 else None, m, 1, None)
        for l in range(1, upto + 1):
            src = ws.r1 if l == 1 else ws.buf[(l - 2) % 2]
            dst = ws.sums if l == 5 else ws.buf[(l - 1) % 2]
            o.x3_layer(l, src, dst, model.wfrag[l], 0, model.bias[l], model.wscale[l], 0, ws.aff[l - 1],
                       0 if l == 1 else 2 * CH[l], ws.stats[l] if l == stats_layer else None, m, 1, l == 1,
                       thr[l - 1], thr[l], seed, pb, int(window_offset) + s, 0, None, None, None, ws.gscale[l - 1],
                       *_sign(l, sl))

    def finish_layer(l: int, repeat: int) -> None:
        if sync is not None:
            _sync_stats(sync, ws.stats[l], 1, CH[l + 1])
        g, b, mm, mv = model.bn[l]
        o.x3_aff(ws.stats[l], g, b, mm, mv, ws.aff[l], CH[l + 1], 1, 0, bool(update_moving), repeat, inv_count, eps,
                 mom, dsc[l], None, ws.gscale[l])

    # block 1: no dropout before it, so its moments (and affine) are shared by every pass
    ws.stats[0].zero_()
    for s, e in bounds:
        run(s, e, 0, int(pass_base), 0)
    finish_layer(0, n_pass)
    for t in range(n_pass):
        pb = int(pass_base) + t
        for l in range(1, 6):
            ws.stats[l].zero_()
            for s, e in bounds:
                run(s, e, l, pb, l)
            finish_layer(l, 1)
        for s, e in bounds:
            run(s, e, 5, pb, -1)
            o.x3_head(ws.sums, ws.aff[5], 0, model.dw, model.db, 0, ws.out, e - s, 1, False)
            out[t, s:e].copy_(ws.out[: e - s])
    return out


@torch.no_grad()
def forward_running(model: X3Model, x: torch.Tensor, n_pass: int = 1, dropout: bool = False, seed: int = 0,
                    pass_offset: int = 0, window_offset: int = 0, logits: bool = False,
                    max_samples: Optional[int] = None) -> torch.Tensor:
    """BN on moving statistics, fp32-faithful: (G, n_pass, N) probabilities (or logits).

    G > 1 members run as one launch per layer (Deep Ensemble predict, ``uq_techniques.py:29``);
    ``dropout=True`` is standard MC Dropout with n_pass passes (one model).  Windows are independent
    here, so sets larger than the activation budget (``max_samples`` window x group rows) run in window
    chunks.  With ``dropout=True`` the result does not depend on the chunking, bitwise (masks are keyed
    by the global window id and the range-safe prescale is per sample).  The Deep-Ensemble path
    (``dropout=False``, :func:`_predict_members`) picks its prescale per member and block from the whole
    launch's sums of squares, so a window's fp16 split -- and with it the last bits of its result -- can
    depend on the other windows of its chunk: results of different chunkings agree to ~1e-7 in
    probability, not bitwise (``tests/test_x3_gpu.py::test_de_chunking_and_float64_large``)."""
    x = x.to(device=model.device, dtype=torch.float32).contiguous()
    n = x.shape[0]
    groups = (n_pass if dropout else model.G) if n > 0 else 1
    if max_samples is None:
        max_samples = _max_samples(model.device, BYTES_PER_SAMPLE + R1_BYTES)
    wc = max(1, int(max_samples) // max(groups, 1))
    if n <= wc:
        return _forward_running(model, x, n_pass, dropout, seed, pass_offset, window_offset, logits)
    parts = [_forward_running(model, x[s: s + wc], n_pass, dropout, seed, pass_offset, int(window_offset) + s, logits)
             for s in range(0, n, wc)]
    return torch.cat(parts, dim=2)


def _forward_running(model: X3Model, x: torch.Tensor, n_pass: int, dropout: bool, seed: int, pass_offset: int,
                     window_offset: int, logits: bool) -> torch.Tensor:
    spec, o = model.spec, _ops()
    n = x.shape[0]
    G = model.G
    if dropout and G != 1:
        raise ValueError("MC Dropout runs one model")
    if not dropout:
        n_pass = 1
    groups = n_pass if dropout else G
    ws = model.workspace(groups * n, n * G, max(groups, G))
    thr = [rng.dropout_threshold(b.dropout) if dropout else 0 for b in spec.blocks]
    dsc = [_dsc(b.dropout) if dropout else 1.0 for b in spec.blocks]
    eps, mom = float(spec.bn_epsilon), float(spec.bn_momentum)
    seed = int(seed) & ((1 << 63) - 1)
    if not dropout:
        return _predict_members(model, ws, x, G, eps, mom, logits)
    sl = _sign_layers()
    # BN affine of the moving statistics, per member (shared by all passes with dropout)
    for l in range(6):
        g, b, mm, mv = model.bn[l]
        o.x3_aff(None, g, b, mm, mv, ws.aff[l], CH[l + 1], G, CH[l + 1] if G > 1 else 0, False, 1, 1.0, eps, mom,
                 dsc[l], ws.amax[l])
    o.x3_l1(x, model.w1, model.b1, ws.r1, None, n, G, ws.smax[0])
    per_member = G > 1
    for l in range(1, 6):
        src = ws.r1 if l == 1 else ws.buf[(l - 2) % 2]
        dst = ws.sums if l == 5 else ws.buf[(l - 1) % 2]
        wstride = model.wfrag[l].shape[1] // 8 if per_member else 0
        sm = ws.smax_out(l, groups * n)
        o.x3_layer(l, src, dst, model.wfrag[l], wstride, model.bias[l], model.wscale[l],
                   CH[l + 1] if per_member else 0, ws.aff[l - 1], 2 * CH[l] if per_member else 0, None, n, groups,
                   dropout and l == 1, thr[l - 1], thr[l], seed, int(pass_offset),
                   int(window_offset), 0, ws.smax[l - 1], ws.amax[l - 1], sm, None, *_sign(l, sl))
    o.x3_head(ws.sums, ws.aff[5], 2 * CH[6] if per_member else 0, model.dw, model.db, CH[6] if per_member else 0,
              ws.out, n, groups, bool(logits))
    return ws.out[: groups * n].view(G, n_pass, n).clone()


# ------------------------------------------------------------------------------------------------
# CPU emulation of the engine's arithmetic from the packed fragments (fp32 conv of hi + lo weights,
# activations split the same way): validates the packing on the CPU tier.
# ------------------------------------------------------------------------------------------------
def _predict_members(model: X3Model, ws: "_Workspace", x: torch.Tensor, G: int, eps: float, mom: float,
                     logits: bool) -> torch.Tensor:
    """Deep-Ensemble predict (``uq_techniques.py:29``): BN on each member's moving statistics, every member
    in one launch per layer.  The staged activations' range-safe prescale is one power of two per member
    and block, bounded by the block output's sums of squares (max R_c <= sqrt(sum R_c^2): the moment
    epilogue of the batch-statistics kernels, used here for the bound only) -- the layer kernels of the
    MC-Dropout phase, no per-sample maximum tracking (2.5 % of the phase).

    Tolerance, not invariance: the bound is taken over every row of the launch, so it can overshoot a
    window's own maximum by up to sqrt(rows) (~2^10 at 16384 windows).  An exact power of two commutes
    with fp16 rounding while both halves stay normal; what the overshoot changes is that the lo halves of
    a window's smallest activations (below ~2^-14 of the chunk's bound) become fp16 subnormals and lose
    their last bits.  Those activations are < 2^-10 of the largest term of their dot products, so the
    effect on a probability is ~1e-7 (measured: chunked vs one launch, and against float64 at 4096
    windows, ``tests/test_x3_gpu.py::test_de_chunking_and_float64_large``); the per-sample prescale of the
    dropout path is bitwise chunk-invariant instead."""
    spec, o = model.spec, _ops()
    n = x.shape[0]
    per_member = G > 1
    ps = CH[1:] if per_member else [0] * 6
    o.zero_buffers([ws.stats[l][: G * STAT_SLOTS * 2 * CH[l + 1]] for l in range(5)])
    g, b, mm, mv = model.bn[5]  # block 6 feeds the fp32 head: no prescale
    o.x3_aff(None, g, b, mm, mv, ws.aff[5], CH[6], G, ps[5], False, 1, 1.0, eps, mom, 1.0, None)
    o.x3_l1(x, model.w1, model.b1, ws.r1, ws.stats[0], n, G, None)
    for l in range(1, 6):
        g, b, mm, mv = model.bn[l - 1]
        o.x3_aff(ws.stats[l - 1], g, b, mm, mv, ws.aff[l - 1], CH[l], G, ps[l - 1], False, 1, 1.0, eps, mom, 1.0,
                 None, ws.gscale[l - 1], True)
        src = ws.r1 if l == 1 else ws.buf[(l - 2) % 2]
        dst = ws.sums if l == 5 else ws.buf[(l - 1) % 2]
        wstride = model.wfrag[l].shape[1] // 8 if per_member else 0
        o.x3_layer(l, src, dst, model.wfrag[l], wstride, model.bias[l], model.wscale[l], ps[l],
                   ws.aff[l - 1], 2 * CH[l] if per_member else 0, ws.stats[l] if l < 5 else None, n, G, False, 0, 0,
                   0, 0, 0, 0, None, None, None, ws.gscale[l - 1], False, False)
    o.x3_head(ws.sums, ws.aff[5], 2 * CH[6] if per_member else 0, model.dw, model.db, CH[6] if per_member else 0,
              ws.out, n, G, bool(logits))
    return ws.out[: G * n].view(G, 1, n).clone()


def split_f16(a: torch.Tensor):
    hi = a.half()
    lo = (a - hi.float()).half()
    return hi, lo


def emulate_conv(h: torch.Tensor, fr: torch.Tensor, wscale: float, k: int, cin: int, cout: int) -> torch.Tensor:
    """The x3 product of one layer in float64: (hi+lo of h) conv (hi+lo of W) minus the lo*lo term."""
    from ..models.reference import conv1d_same

    nch, nct = cin // CK, cout // 16
    v = fr.reshape(nch, k, nct, 2, 4, 16, 8).double()
    whi = v[:, :, :, 0].permute(1, 0, 3, 5, 2, 4).reshape(k, cin, cout)
    wlo = v[:, :, :, 1].permute(1, 0, 3, 5, 2, 4).reshape(k, cin, cout)
    ah, al = split_f16(h.float())
    ah, al = ah.double(), al.double()
    z = torch.zeros(cout, dtype=torch.float64)
    y = conv1d_same(ah, whi, z) + conv1d_same(ah, wlo, z) + conv1d_same(al, whi, z)
    return y * wscale
