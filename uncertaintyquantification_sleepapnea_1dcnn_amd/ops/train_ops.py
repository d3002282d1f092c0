"""Host orchestration of the layer-wise HIP training kernels (``csrc/train_conv.hip``).

One optimizer step (Keras semantics) is ~22 launches on one stream:

  pack (bf16 MFMA fragments of all 6 kernels, forward + dgrad orientation)
  fwd 1..6          R_l = relu(conv(dropout(BN(R_{l-1}))) + b), per-channel moments (atomics)
  head              GAP + Dense + BCE + dlogit + dense grads + backward moments of block 6
  dgrad 6..2        dY_{l-1} and the backward moments of block l-1
  wgrad 6..1        dW_l, db_l (row-reduced in registers, per-row-group partial slots + ordered reduce)
  finalize          moving-average update + dgamma / dbeta
  Adam              one multi-tensor launch over the flat buffer

With data parallelism (``sync``) the per-layer moments and the backward moments are all-reduced
between the launches (SyncBN: exactly the full-batch statistics of the reference's single-device
Keras BN) and the flat gradient once at the end (one bucket, C1).

The same forward kernels with ``groups = T`` implement MC Dropout with BatchNorm on per-pass
batch statistics over the whole test set (the reference's ``model(x, training=True)``, Q1).
"""
from __future__ import annotations

import os
import struct
from typing import Callable, List, Optional

import numpy as np
import torch

from ..models.spec import ModelSpec
from . import _ext, fused, rng

SR, HALO, ROWS_PER_TILE = 64, 4, 128
TRAIN_PASS_BASE = 1 << 30
STAT_SLOTS = 16  # must equal kStatSlots in csrc/train_conv.hip


def supports(spec: ModelSpec) -> bool:
    """True if the HIP training kernels implement ``spec``.  On a GPU machine a missing extension
    raises (no silent eager fallback) unless ``APNEAUQ_ALLOW_FALLBACK=1``."""
    if not fused.supports(spec):
        return False
    if _ext.available():
        return True
    if not _ext.fallback_allowed():
        _ext.require()
    return False


def _fbits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]


def padded_rows(n_samples: int) -> int:
    return ROWS_PER_TILE * ((n_samples + 1) // 2) + 2 * HALO


def to_padded(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(N, 60, C) -> padded-row layout (rows, C) bf16 with zero pad rows."""
    n, L, c = x.shape
    if out is None:
        out = torch.zeros(padded_rows(n), c, dtype=torch.bfloat16, device=x.device)
    out[HALO: HALO + SR * n].view(n, SR, c)[:, :L].copy_(x)
    return out


class TrainWorkspace:
    """Device buffers + pointer context for one model and one (max) batch size."""

    def __init__(self, model, batch: int, groups: int = 1, n_win: Optional[int] = None, with_backward: bool = True,
                 shared0: bool = False, deterministic: bool = False):
        spec = model.spec
        store = model.store
        dev = store.device
        self.model = model
        self.B = int(batch)
        self.groups = int(groups)
        self.n_win = int(n_win if n_win is not None else batch)
        # shared0 (batch-BN MC Dropout): the input and block 1's output exist once per window
        self.shared0 = bool(shared0)
        rows = padded_rows(self.B)
        rows0 = padded_rows(self.n_win) if self.shared0 else rows
        ch = spec.channels()
        ks = [b.kernel_size for b in spec.blocks]
        bf = torch.bfloat16
        self.x = torch.zeros(rows0, ch[0], dtype=bf, device=dev)
        # -0.0 everywhere: the halo rows before the first / after the last tile and the 4 pad rows of
        # every sample are never written by the kernels (train_conv.hip copy-out of the valid rows), and -0.0
        # decodes to A = 0 (decode_pair) like a dropped element
        self.R = [torch.empty(rows0 if l == 0 else rows, ch[l + 1], dtype=bf, device=dev).fill_(-0.0)
                  for l in range(6)]
        self.dY = [torch.zeros(rows, ch[l + 1], dtype=bf, device=dev) if (with_backward and l < 5)
                   else torch.zeros(16, dtype=bf, device=dev) for l in range(6)]
        # dZ_l materialised by dgrad_l for wgrad_l (block 1 has no dgrad)
        self.dZ = [torch.zeros(rows, ch[l + 1], dtype=bf, device=dev) if (with_backward and l >= 1)
                   else torch.zeros(16, dtype=bf, device=dev) for l in range(6)]
        # BN moment sums: STAT_SLOTS interleaved copies per layer (kernels add into slot wg % S and
        # readers sum the slots; train_conv.hip kStatSlots) -> st[S][groups][2][C], bst[S][2][C] (fp64)
        S = STAT_SLOTS
        self.st_all = torch.zeros(sum(S * self.groups * 2 * ch[l + 1] for l in range(6)), dtype=torch.float64,
                                  device=dev)
        self.bst_all = torch.zeros(sum(S * 2 * ch[l + 1] for l in range(6)), dtype=torch.float64, device=dev)
        self.st, self.bst = [], []
        o1 = o2 = 0
        for l in range(6):
            n1, n2 = S * self.groups * 2 * ch[l + 1], S * 2 * ch[l + 1]
            self.st.append(self.st_all[o1: o1 + n1])
            self.bst.append(self.bst_all[o2: o2 + n2])
            o1 += n1
            o2 += n2
        self.wf, self.wd = [], []
        for l in range(6):
            nf = ((ch[l] * ks[l] + 31) // 32) * 32 * ch[l + 1]
            nd = ((ch[l + 1] * ks[l] + 31) // 32) * 32 * ch[l]
            self.wf.append(torch.zeros(nf, dtype=bf, device=dev))
            self.wd.append(torch.zeros(nd, dtype=bf, device=dev))
        # wgrad partials (one slot per row group, summed in order by wgrad_reduce: deterministic and
        # cheaper than fp32 atomics); shared by the six sequential wgrad launches
        self.wpart = (torch.empty(int(_ext.ops().train_wgrad_part_size(self.B)), device=dev)
                      if with_backward else None)
        # deterministic mode: per-workgroup / per-sample partials of the BN moments, head and dgrad
        # sums, added in a fixed order by det_reduce_kernel instead of atomics (training only)
        self.deterministic = bool(deterministic) and with_backward and self.groups == 1 and not self.shared0
        self.det = (torch.empty(int(_ext.ops().train_det_size(self.B)), device=dev) if self.deterministic else None)
        # single-device training: per-layer BN parameter table, written once per step after the
        # forward kernels (train_conv.hip Args::tab / tab_kernel)
        self.tab = torch.zeros(6 * 6 * 256, device=dev) if with_backward else None
        # training head: slotted dense-weight / loss / dense-bias sums (train_conv.hip Args::hpart)
        self.hpart = torch.zeros(STAT_SLOTS * (ch[6] + 2), device=dev) if with_backward else None
        self.y = torch.zeros(self.B, device=dev)
        self.logits = torch.zeros(self.B, device=dev)
        self.dlogit = torch.zeros(self.B, device=dev)
        self.loss = torch.zeros(1, device=dev)
        self.grad = torch.zeros_like(store.flat)
        self.gviews = {}
        for n in store.trainable:
            off = store.offsets[n]
            self.gviews[n] = self.grad[off: off + store.views[n].numel()].view(store.shapes[n])
        self.ks = ks
        self.ch = ch
        self._ctx_key = None
        self.ctx = None
        # [dropout pass offset, Adam iterations] on the device: read by the kernels when the step
        # is replayed from a captured HIP graph (see GraphedTrainStep)
        self.counters = torch.zeros(2, dtype=torch.int32, device=dev)

    def build_ctx(self, n: int, n_win: int, groups: int, window_offset: int, seed: int, dropout: bool,
                  inv_count: float, inv_batch: float, device_counters: bool = False, table: bool = False):
        """``table``: the kernels exchange BN parameters through ``self.tab`` (single device, one stats
        group, atomic mode only -- synchronised / deterministic moments are only final after the
        kernel that produces them)."""
        table = bool(table) and self.tab is not None and groups == 1 and self.det is None
        key = (n, n_win, groups, window_offset, seed, dropout, inv_count, inv_batch, device_counters, table)
        if key == self._ctx_key:
            return self.ctx
        spec, v, g = self.model.spec, self.model.store.views, self.gviews
        vals: List[int] = []
        for l in range(6):
            i = l + 1
            p = spec.blocks[l].dropout
            vals += [self.wf[l].data_ptr(), self.wd[l].data_ptr(), v[f"conv1d_{i}/bias"].data_ptr(),
                     v[f"batchnorm_{i}/gamma"].data_ptr(), v[f"batchnorm_{i}/beta"].data_ptr(),
                     v[f"batchnorm_{i}/moving_mean"].data_ptr(), v[f"batchnorm_{i}/moving_variance"].data_ptr(),
                     g[f"conv1d_{i}/kernel"].data_ptr(), g[f"conv1d_{i}/bias"].data_ptr(),
                     g[f"batchnorm_{i}/gamma"].data_ptr(), g[f"batchnorm_{i}/beta"].data_ptr(),
                     self.R[l].data_ptr(), self.dY[l].data_ptr(), self.st[l].data_ptr(), self.bst[l].data_ptr(),
                     rng.dropout_threshold(p), _fbits(1.0 / (1.0 - p) if p < 1 else 0.0), self.dZ[l].data_ptr()]
        vals += [self.x.data_ptr(), self.y.data_ptr(), v["output_layer/kernel"].data_ptr(),
                 v["output_layer/bias"].data_ptr(), g["output_layer/kernel"].data_ptr(),
                 g["output_layer/bias"].data_ptr(), self.logits.data_ptr(), self.dlogit.data_ptr(),
                 self.loss.data_ptr(), n, n_win, groups, TRAIN_PASS_BASE, window_offset,
                 int(seed) & ((1 << 63) - 1), int(bool(dropout)), _fbits(inv_count), _fbits(inv_batch),
                 _fbits(spec.bn_epsilon), _fbits(spec.bn_momentum),
                 self.counters.data_ptr() if device_counters else 0, self.groups, int(self.shared0),
                 self.wpart.data_ptr() if self.wpart is not None else 0,
                 self.det.data_ptr() if self.det is not None else 0,
                 self.tab.data_ptr() if table else 0,
                 self.hpart.data_ptr() if (self.hpart is not None and self.det is None) else 0]
        self.ctx = torch.tensor(vals, dtype=torch.int64)
        self._ctx_key = key
        return self.ctx

    def pack(self) -> None:
        """bf16 MFMA fragments of all six conv kernels (forward + dgrad orientation) in ONE launch
        (csrc/generic_wgrad.hip pack_kernel: the same fragment layout as train_conv.hip's per-layer
        pack for channel counts that are multiples of 16; block 1 has no dgrad)."""
        v = self.model.store.views
        if not hasattr(self, "_no_dgr"):
            self._no_dgr = torch.empty(0, dtype=torch.bfloat16, device=self.wf[0].device)
        _ext.ops().gt_pack([v[f"conv1d_{l + 1}/kernel"] for l in range(6)], self.wf,
                           [self._no_dgr] + self.wd[1:], self.ks, self.ch[:6], self.ch[1:])

    def accumulators(self) -> List[torch.Tensor]:
        """BN moment / backward sums, the flat gradient, the loss (and the head's slots)."""
        return [self.st_all, self.bst_all, self.grad, self.loss] + ([self.hpart] if self.hpart is not None else [])

    def zero_accumulators(self) -> None:
        """The accumulators: one launch."""
        _ext.ops().zero_buffers(self.accumulators())

    def pack_args(self):
        v = self.model.store.views
        if not hasattr(self, "_no_dgr"):
            self._no_dgr = torch.empty(0, dtype=torch.bfloat16, device=self.wf[0].device)
        return ([v[f"conv1d_{l + 1}/kernel"] for l in range(6)], list(self.wf), [self._no_dgr] + self.wd[1:],
                list(self.ks), list(self.ch[:6]), list(self.ch[1:]))

    def pack_zero(self) -> None:
        """:meth:`pack` and :meth:`zero_accumulators` as ONE launch (the graphed step's first node)."""
        _ext.ops().gt_pack_zero(*self.pack_args(), self.accumulators())


def _inputs_direct(xs, ys, n: int, dev: torch.device, cin: int) -> bool:
    """The fused input copy applies: fp32 contiguous (n, 60, cin) windows and (n,) labels, already on the
    workspace's device (the kernel reads them in place).  Anything else -- CPU batches, another device,
    another channel count -- takes the ``copy_`` path, which moves or rejects it."""
    return all(x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 3 and x.shape[0] == n and
               x.shape[1] == 60 and x.shape[2] == cin and x.is_cuda and x.device == dev for x in xs) and \
        all(y.dtype == torch.float32 and y.is_contiguous() and y.numel() == n and y.is_cuda and y.device == dev
            for y in ys)


def _call(ctx, op, layer=0, flag=0, pass_base=-1, device=0):
    _ext.ops().train_call(ctx, op, layer, flag, pass_base, device)


# Deterministic training: every reduction of the HIP training step in a fixed order, so
# two runs give bitwise-identical weights.  APNEAUQ_DETERMINISTIC=1 or set_deterministic(True);
# costs a few small reduce launches per step.
DETERMINISTIC = os.environ.get("APNEAUQ_DETERMINISTIC", "0") not in ("", "0")
# GraphedTrainStep: dgrad and wgrad chains on two captured streams (APNEAUQ_TRAIN_OVERLAP=1).  Off by
# default: the chains do run concurrently (34 % of kernel time overlapped at batch 1024) but each
# kernel already holds every CU, so both slow ~2x and the step got slower (0.76 -> 0.82 ms at batch
# 1024, 4.37 -> 4.51 ms at 8192; profiles/train_step_r4.md)
OVERLAP = os.environ.get("APNEAUQ_TRAIN_OVERLAP", "0") not in ("", "0")
# Fused reductions (single-device atomic-mode steps): wgrad_l's partial sums are reduced by the workgroups
# of dgrad_{l-1} as they finish their tiles, those of wgrad_1 / wgrad_0 by one launch with the BN finalize
# -- 7 reduce / finalize launches become 1 (csrc/train_conv.hip train_launch_dgrad / _finalize; the same
# column split and summation order, so the gradients equal the separate reduces' bitwise).  Up to
# FUSED_MAX_BATCH samples: dgrad's 8 waves per CU run the reduction latency-bound, ~2x the reduce
# launch's time, which only the launch overhead saved at small batches pays for (batch 1024: -13 us of
# kernel time per step; batch 8192: +16 us; profiles/train_fused_reduce_r6.md).
# APNEAUQ_TRAIN_FUSED_REDUCE=0 restores the separate launches.
FUSED_REDUCE = os.environ.get("APNEAUQ_TRAIN_FUSED_REDUCE", "1") not in ("", "0")
FUSED_MAX_BATCH = int(os.environ.get("APNEAUQ_TRAIN_FUSED_MAX_BATCH", "2048"))


def set_deterministic(flag: bool = True) -> None:
    global DETERMINISTIC
    DETERMINISTIC = bool(flag)


def _get_ws(model, batch: int) -> TrainWorkspace:
    ws = getattr(model, "_train_ws", None)
    if ws is None or ws.B < batch or ws.groups != 1 or ws.deterministic != DETERMINISTIC:
        ws = TrainWorkspace(model, batch, deterministic=DETERMINISTIC)
        model._train_ws = ws
    return ws


def train_step(model, x: torch.Tensor, y: torch.Tensor, grad_allreduce=None, sync: Optional[Callable] = None,
               global_batch: Optional[int] = None, window_offset: int = 0, sync_world: int = 1):
    """One Keras-semantics optimizer step with the HIP kernels; returns (loss_sum, probs).

    ``sync`` (data parallel, ``sync_world`` ranks) all-reduces the BN moments and backward sums, so
    the dgamma / dbeta the finalize writes are already global; they are pre-divided by
    ``sync_world`` because ``grad_allreduce`` sums the whole flat gradient once more.
    """
    n = x.shape[0]
    ws = _get_ws(model, n)
    gb = global_batch or n
    ctx = ws.build_ctx(n, n, 1, window_offset, model.seed, True, 1.0 / (gb * 60), 1.0 / gb, table=sync is None)
    dev = x.device.index or 0
    # inputs in padded-row layout (pad rows stay zero)
    ws.x[HALO: HALO + SR * n].view(n, SR, ws.ch[0])[:, :60].copy_(x)
    if n < ws.B:  # a partial last batch: clear rows of samples beyond n (stale data from a larger batch)
        ws.x[HALO + SR * n:].zero_()
    ws.y[:n].copy_(y.reshape(-1))
    ws.zero_accumulators()
    ws.pack()
    pb = TRAIN_PASS_BASE + model._train_step_counter
    for l in range(6):
        _call(ctx, 0, l, 0, pb, dev)
        if sync is not None:
            sync(ws.st[l])
    _call(ctx, 1, 0, 3, pb, dev)  # head + the BN parameter table's forward rows (no-op without a table)
    if sync is not None:
        sync(ws.bst[5])
        for l in range(5, 0, -1):
            _call(ctx, 2, l, 0, pb, dev)
            sync(ws.bst[l - 1])
            _call(ctx, 3, l, 0, pb, dev)
        _call(ctx, 3, 0, 0, pb, dev)
        _call(ctx, 4, 1, 1, pb, dev)
    else:
        _backward_calls(ctx, pb, dev, _fused(ws, n))
    if sync is not None and sync_world > 1:
        for i in range(1, 7):
            ws.gviews[f"batchnorm_{i}/gamma"].div_(sync_world)
            ws.gviews[f"batchnorm_{i}/beta"].div_(sync_world)
    scale = 1.0
    if grad_allreduce is not None:
        scale = grad_allreduce(ws.grad)
    # device-side bias correction, as the captured step computes it (eager == graph bitwise)
    model.optimizer.step(model.store.flat, ws.grad, grad_scale=scale, counters=ws.counters)
    return ws.loss.double().sum(), torch.sigmoid(ws.logits[:n])


def _fused(ws, n: int) -> bool:
    """A step of n samples runs the fused reductions: atomic mode with the parameter table (single
    device), at most FUSED_MAX_BATCH samples."""
    return FUSED_REDUCE and n <= FUSED_MAX_BATCH and ws.tab is not None and ws.det is None and ws.wpart is not None


def _backward_calls(ctx, pb, dev, fused: bool) -> None:
    """dgrad_l, wgrad_l for l = 5..1, wgrad_0, finalize -- the eager step and the captured graph issue
    the same launches.  fused: no reduce launches; dgrad_l (l <= 4) reduces wgrad_{l+1}'s partials and the
    finalize launch those of wgrad_1 and wgrad_0."""
    f = 2 if fused else 0
    for l in range(5, 0, -1):
        _call(ctx, 2, l, f if l < 5 else 0, pb, dev)
        _call(ctx, 3, l, f, pb, dev)
    _call(ctx, 3, 0, f, pb, dev)
    _call(ctx, 4, 1, 1 | f, pb, dev)


def capture_graph(body, dev):
    """Capture ``body()`` (HIP launches only) as a graph on a side stream.

    A garbage collection during the capture can destroy an OLD graph, which HIP refuses while a stream
    is capturing (abort), so collection is paused.  The device is synchronised once after the capture
    (a one-time cost per graph): the stale first-replay inputs once seen on the generic path (round 2:
    ~1 in 40 captures) came with a per-step host-written dropout-key array that the steps no longer
    use (keys are derived on the device from the counters, ``stream_keys``; 40 + 40 fresh captures of
    the single-model paths replayed correctly without it, ``profiles/capture_race_r3.txt``), but the
    member-batched capture (multi-stream groups, a device Args array uploaded right before capture)
    was never probed, so the synchronize stays on.  ``APNEAUQ_CAPTURE_SYNC=0`` drops it."""
    import gc

    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph, stream=side):
                body()
    finally:
        if was:
            gc.enable()
    torch.cuda.current_stream(dev).wait_stream(side)
    if os.environ.get("APNEAUQ_CAPTURE_SYNC", "1") != "0":
        torch.cuda.synchronize(dev)
    return graph


def bound_key(model):
    """What a captured training graph bakes in: buffer identities and the optimizer's scalars
    (learning rate / betas / epsilon are kernel arguments of the captured Adam launch)."""
    opt = model.optimizer
    return (model.store.flat, opt.m, opt.v, float(opt.learning_rate), float(opt.beta_1), float(opt.beta_2),
            float(opt.epsilon))


def _same_bound(a, b) -> bool:
    return all(x is y for x, y in zip(a[:3], b[:3])) and tuple(a[3:]) == tuple(b[3:])


class GraphedTrainStep:
    """The whole HIP training step of one batch size captured once as a HIP graph and replayed.

    At batch 128-256 the eager step is bound by ~25 kernel launches + ~20 small tensor ops issued
    from Python (~0.8 ms/step whatever the batch); a replay is one graph launch.  The dropout pass id
    and Adam's bias-correction step come from the workspace's device counters, bumped by the last
    node of the graph, so replays are exactly the steps the eager path would run (the host mirrors
    ``model._train_step_counter`` / ``optimizer.iterations`` advance in lockstep and the device
    counters are re-synced if they were changed outside, e.g. by an eager step or a restore).
    Single device only (a data-parallel step all-reduces through torch.distributed).
    """

    def __init__(self, model, batch: int):
        self.model = model
        self.batch = int(batch)
        dev = model.store.device
        self.ws = TrainWorkspace(model, self.batch, deterministic=DETERMINISTIC)
        self.deterministic = DETERMINISTIC
        n = self.batch
        # the step's inputs are copied straight into the workspace's padded-row buffers (views; the
        # pad rows stay zero), outside the graph: no copy nodes inside it
        self.x_in = self.ws.x[HALO: HALO + SR * n].view(n, SR, self.ws.ch[0])[:, :60]
        self.y_in = self.ws.y[:n]
        self.probs = torch.empty(n, dtype=torch.float32, device=dev)
        self.ctx = self.ws.build_ctx(n, n, 1, 0, model.seed, True, 1.0 / (n * 60), 1.0 / n, device_counters=True,
                                     table=True)
        model.optimizer._ensure(model.store.flat)
        # the graph bakes these buffers' addresses: a replay is only valid while they are the same
        # tensor objects (a restored optimizer state or a moved model triggers a re-capture)
        self.bound = bound_key(model)
        self._sync_counters()
        # wgrad chain on a second captured stream (see _body); needs the parameter table
        self.overlap = OVERLAP and self.ws.tab is not None and not self.deterministic
        self.aux = torch.cuda.Stream(dev) if self.overlap else None
        outs = []
        self.graph = capture_graph(lambda: outs.extend(self._body()), dev)
        self.loss_out, self.probs_out = outs

    def _state(self):
        return (int(self.model._train_step_counter), int(self.model.optimizer.iterations))

    def _sync_counters(self):
        st = self._state()
        self.ws.counters.copy_(torch.tensor(st, dtype=torch.int32))
        self._dev_state = st

    def _body(self):
        ws, n, o = self.ws, self.batch, _ext.ops()
        dev = self.x_in.device.index or 0
        ws.pack_zero()
        for l in range(6):
            _call(self.ctx, 0, l, 0, TRAIN_PASS_BASE, dev)
        _call(self.ctx, 1, 0, 3, TRAIN_PASS_BASE, dev)  # head + the BN parameter table's forward rows
        if self.overlap:
            # wgrad_l needs only dgrad_l's dZ_l (and forward state), and no dgrad reads a wgrad
            # output: the wgrad + reduce chain runs on its own stream, forked after each dgrad and
            # joined before the finalize / Adam (measured slower, see OVERLAP).  Both sum the backward
            # BN rows from the slots (flag 1) -- the table rows come from the reduces' side job, which
            # would tie dgrad_{l-1} to wgrad_l again.
            main, aux = torch.cuda.current_stream(), self.aux
            self._evs = []  # alive for the capture
            for l in range(5, 0, -1):
                _call(self.ctx, 2, l, 1, TRAIN_PASS_BASE, dev)
                ev = torch.cuda.Event()
                self._evs.append(ev)
                ev.record(main)
                aux.wait_event(ev)
                with torch.cuda.stream(aux):
                    _call(self.ctx, 3, l, 1, TRAIN_PASS_BASE, dev)
            with torch.cuda.stream(aux):
                _call(self.ctx, 3, 0, 1, TRAIN_PASS_BASE, dev)
            ev = torch.cuda.Event()
            self._evs.append(ev)
            ev.record(aux)
            main.wait_event(ev)
            _call(self.ctx, 4, 1, 1, TRAIN_PASS_BASE, dev)
        else:
            _backward_calls(self.ctx, TRAIN_PASS_BASE, dev, _fused(ws, n))
        opt = self.model.optimizer
        o.adam_step(self.model.store.flat, ws.grad, opt.m, opt.v, opt.beta_1, opt.beta_2, opt.learning_rate,
                    opt.epsilon, 1.0, ws.counters)
        o.train_tail(ws.counters, [ws.logits[:n]], [self.probs])  # counters + 1, probs: one node
        # the loss sum as a 0-d view of the kernels' fp32 accumulator (no cast / reduce nodes)
        return ws.loss.view(()), self.probs

    def __call__(self, x: torch.Tensor, y: torch.Tensor):
        """One step; returns (loss_sum, probs) views of static buffers (valid until the next replay)."""
        if self._state() != self._dev_state:
            self._sync_counters()
        yf = y.reshape(-1)
        if _inputs_direct([x], [yf], self.batch, self.ws.x.device, self.ws.ch[0]):  # both copies in one launch
            _ext.ops().train_inputs([x], [yf], [self.ws.x[HALO:]], [self.ws.y], SR)
        else:
            self.x_in.copy_(x)
            self.y_in.copy_(yf)
        self.graph.replay()
        self.model.optimizer.iterations += 1
        self._dev_state = (self._dev_state[0] + 1, self._dev_state[1] + 1)
        return self.loss_out, self.probs_out


def graph_train_step(model, x: torch.Tensor, y: torch.Tensor):
    """Replay (capturing on first use) the graphed step for this batch size."""
    g = getattr(model, "_train_graphs", None)
    if g is None:
        g = model._train_graphs = {}
    n = int(x.shape[0])
    opt = model.optimizer
    cur = g.get(n)
    if cur is None or not _same_bound(cur.bound, bound_key(model)) or cur.deterministic != DETERMINISTIC:
        g[n] = cur = GraphedTrainStep(model, n)
    return cur(x, y)


class GraphedEnsembleStep:
    """One optimizer step of M ensemble members (same architecture and batch size, one GPU) as ONE
    captured HIP graph whose layer kernels are member-batched: every forward / head / dgrad / wgrad /
    finalize launch covers all members (``gridDim.z = M``, each member's pointers from a device array
    of kernel arguments, ``csrc/train_conv.hip:train_launch_mb``).  A batch-1024 step of this CNN is
    ~500 workgroups per launch -- one round on 256 CUs with its memory phases exposed back to back --
    so stacking the members in one launch fills the machine instead of overlapping them on streams
    (``training/trainer.py:fit_concurrent``).  Per member the step is exactly
    :class:`GraphedTrainStep`'s: own workspace, dropout step and Adam counters (bumped in the graph),
    own weights and optimizer state; replaces the reference's sequential member loop
    (``train_deep_ensemble_cnns.py:125-177``)."""

    def __init__(self, models, batch: int):
        self.models = list(models)
        self.batch = n = int(batch)
        M = len(self.models)
        if M < 1:
            raise ValueError("GraphedEnsembleStep needs at least one member")
        dev = self.models[0].store.device
        if any(m.store.device != dev for m in self.models):
            raise ValueError("ensemble members must share one device")
        self.ws, self.ctx, self.x_in, self.y_in = [], [], [], []
        # every member's device counters [dropout step, Adam iterations] are rows of one tensor: one bump
        self.counters = torch.zeros(M, 2, dtype=torch.int32, device=dev)
        self.deterministic = DETERMINISTIC
        for i, m in enumerate(self.models):
            ws = TrainWorkspace(m, n, deterministic=self.deterministic)
            ws.counters = self.counters[i]
            self.ws.append(ws)
            self.x_in.append(ws.x[HALO: HALO + SR * n].view(n, SR, ws.ch[0])[:, :60])
            self.y_in.append(ws.y[:n])
            self.ctx.append(ws.build_ctx(n, n, 1, 0, m.seed, True, 1.0 / (n * 60), 1.0 / n, device_counters=True,
                                         table=True))
            m.optimizer._ensure(m.store.flat)
        self.probs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(M)]
        self.args = _ext.ops().train_args_dev(self.ctx, dev.index or 0)
        self.bound = [bound_key(m) for m in self.models]
        self._sync_counters()
        outs = []
        self.graph = capture_graph(lambda: outs.extend(self._body()), dev)
        self.loss_out = outs[:M]
        self.probs_out = outs[M:]

    def _state(self):
        return [(int(m._train_step_counter), int(m.optimizer.iterations)) for m in self.models]

    def _sync_counters(self):
        st = self._state()
        self.counters.copy_(torch.tensor(st, dtype=torch.int32))
        self._dev_state = st

    def _body(self):
        o, M, n = _ext.ops(), len(self.models), self.batch
        # bf16 fragments of every member's six kernels and the members' accumulators cleared: one
        # launch per 8 members (csrc/generic_wgrad.hip pack_kernel: 48 blocks, 48 zero buffers)
        for g0 in range(0, M, 8):
            packs = [ws.pack_args() for ws in self.ws[g0:g0 + 8]]
            o.gt_pack_zero(*[sum((p[i] for p in packs), []) for i in range(6)],
                           sum((ws.accumulators() for ws in self.ws[g0:g0 + 8]), []))
        a, c0 = self.args, self.ctx[0]
        for l in range(6):
            o.train_call_mb(a, c0, M, 0, l, 0)
        o.train_call_mb(a, c0, M, 5, 0, 0)  # BN parameter tables (forward rows)
        o.train_call_mb(a, c0, M, 1, 0, 1)  # head + dlogit + backward sums of block 6
        for l in range(5, 0, -1):
            o.train_call_mb(a, c0, M, 2, l, 0)
            o.train_call_mb(a, c0, M, 3, l, 0)
        o.train_call_mb(a, c0, M, 3, 0, 0)
        o.train_call_mb(a, c0, M, 4, 1, 1)  # moving averages + dgamma / dbeta
        hyper = {(float(m.optimizer.learning_rate), float(m.optimizer.beta_1), float(m.optimizer.beta_2),
                  float(m.optimizer.epsilon)) for m in self.models}
        if len(hyper) == 1:  # one Adam launch per 16 members (csrc/adam.hip kAdamMaxSets)
            lr, b1, b2, eps = hyper.pop()
            for g0 in range(0, M, 16):
                ms, wss = self.models[g0:g0 + 16], self.ws[g0:g0 + 16]
                o.adam_step_multi([m.store.flat for m in ms], [ws.grad for ws in wss], [m.optimizer.m for m in ms],
                                  [m.optimizer.v for m in ms], b1, b2, lr, eps, [ws.counters for ws in wss])
        else:
            for m, ws in zip(self.models, self.ws):
                opt = m.optimizer
                o.adam_step(m.store.flat, ws.grad, opt.m, opt.v, opt.beta_1, opt.beta_2, opt.learning_rate,
                            opt.epsilon, 1.0, ws.counters)
        # every member's counters + 1 and probs = sigmoid(logits): one launch per 32 members
        flat = self.counters.view(-1)
        for g0 in range(0, M, 32):
            o.train_tail(flat[2 * g0: 2 * min(M, g0 + 32)], [ws.logits[:n] for ws in self.ws[g0:g0 + 32]],
                         self.probs[g0:g0 + 32])
        return [ws.loss.view(()) for ws in self.ws] + list(self.probs)

    def valid_for(self, models) -> bool:
        return (len(models) == len(self.models) and all(a is b for a, b in zip(models, self.models)) and
                all(_same_bound(b, bound_key(m)) for b, m in zip(self.bound, self.models)) and
                self.deterministic == DETERMINISTIC)

    def __call__(self, xs, ys):
        """One step of every member on its own batch (lists of (n, 60, 4) / (n,) device tensors);
        returns per-member (loss_sum, probs) views of static buffers (valid until the next replay)."""
        if self._state() != self._dev_state:
            self._sync_counters()
        yfs = [y.reshape(-1) for y in ys]
        M = len(self.models)
        if _inputs_direct(xs, yfs, self.batch, self.ws[0].x.device, self.ws[0].ch[0]):  # one launch per 32 members
            for g0 in range(0, M, 32):
                _ext.ops().train_inputs(list(xs[g0:g0 + 32]), yfs[g0:g0 + 32],
                                        [ws.x[HALO:] for ws in self.ws[g0:g0 + 32]],
                                        [ws.y for ws in self.ws[g0:g0 + 32]], SR)
        else:
            for i in range(M):
                self.x_in[i].copy_(xs[i])
                self.y_in[i].copy_(yfs[i])
        self.graph.replay()
        for m in self.models:
            m.optimizer.iterations += 1
            m._train_step_counter += 1
            m.store.bump()
        self._dev_state = [(a + 1, b + 1) for a, b in self._dev_state]
        return list(zip(self.loss_out, self.probs_out))


def ensemble_supported(models) -> bool:
    """True when :class:`GraphedEnsembleStep` can batch these members: HIP backend on one GPU, the
    reference architecture, single-device training (no data parallelism) and graph replay enabled
    (atomic or deterministic mode: the deterministic member-batched step equals each member's own
    deterministic step bitwise)."""
    if not models or os.environ.get("APNEAUQ_TRAIN_GRAPH", "1") == "0":
        return False
    if os.environ.get("APNEAUQ_TRAIN_BACKEND", "auto") not in ("auto", "hip"):
        return False
    dev = models[0].device
    if dev.type != "cuda":
        return False
    for m in models:
        if m.device != dev or not supports(m.spec) or getattr(m, "dp", None) is not None:
            return False
    return True


def _sync_slots(sync: Callable, st: torch.Tensor, used: int) -> None:
    """SyncBN of one layer's moment buffer: add the STAT_SLOTS interleaved slots locally (fp64), then
    all-reduce the first ``used`` doubles of one slot (16x fewer bytes on the wire than the raw buffer)
    and leave the global sums in slot 0, zeros in the others (the kernels add all slots)."""
    v = st.view(STAT_SLOTS, -1)
    tot = v[:, :used].sum(0)
    sync(tot)
    v[:, :used].zero_()
    v[0, :used].copy_(tot)


@torch.no_grad()
def forward_batch_stats(model, x: torch.Tensor, n_pass: int, pass_base: int, seed: int, update_moving: bool = True,
                        sync: Optional[Callable] = None, window_offset: int = 0, global_n: Optional[int] = None,
                        max_samples: int = 1 << 20) -> torch.Tensor:
    """MC Dropout with BN on per-pass batch statistics (reference semantics): (T, N) probabilities.

    Passes are processed in balanced chunks (statistics are per pass, so chunking is exact).  Block 1
    sees the same input in every pass (no dropout precedes it), so its output and batch moments are
    computed ONCE per call over the N windows and shared by all passes; block 2's staging draws
    block 1's per-pass dropout masks from the counter hash.
    """
    n = x.shape[0]
    gn = global_n or n
    # the chunking must be identical on every rank when ``sync`` all-reduces per chunk: derive it
    # from the largest shard (ceil(global_n / world)) rather than from this rank's n
    ref_n = n
    if sync is not None and global_n:
        import torch.distributed as dist

        w = dist.get_world_size() if dist.is_initialized() else 1
        ref_n = -(-global_n // w)
    cap = max(1, min(n_pass, max_samples // max(ref_n, 1)))
    n_chunks = -(-n_pass // cap)
    chunk = -(-n_pass // n_chunks)  # balanced: e.g. 50 passes at cap 16 -> 13/13/12/12
    outs = []
    dev = x.device.index or 0
    ws = getattr(model, "_mcd_ws", None)
    if ws is None or ws.B != chunk * n or ws.groups != chunk or not ws.shared0 or ws.n_win != n:
        ws = TrainWorkspace(model, chunk * n, groups=chunk, n_win=n, with_backward=False, shared0=True)
        model._mcd_ws = ws
    ws.x[HALO: HALO + SR * n].view(n, SR, ws.ch[0])[:, :60].copy_(x)
    ws.pack()
    for ci, t0 in enumerate(range(0, n_pass, chunk)):
        tc = min(chunk, n_pass - t0)
        bs = tc * n
        ctx = ws.build_ctx(bs, n, tc, window_offset, seed, True, 1.0 / (gn * 60), 1.0)
        if ci == 0:
            ws.st_all.zero_()
            _call(ctx, 0, 0, 1, pass_base + t0, dev)  # block 1 once, over the n windows
            if sync is not None:
                _sync_slots(sync, ws.st[0], 2 * ws.ch[1])  # stats group 0 only
        else:
            ws.st_all[ws.st[0].numel():].zero_()  # block-1 moments stay (they are pass-independent)
        for l in range(1, 6):
            _call(ctx, 0, l, 0, pass_base + t0, dev)
            if sync is not None:
                _sync_slots(sync, ws.st[l], tc * 2 * ws.ch[l + 1])  # the chunk's tc stats groups
        _call(ctx, 1, 0, 0, pass_base + t0, dev)
        if update_moving:
            _call(ctx, 4, 1, 0, pass_base + t0, dev)
        outs.append(torch.sigmoid(ws.logits[:bs].view(tc, n)).clone())
    model.store.bump()
    return torch.cat(outs, 0)
