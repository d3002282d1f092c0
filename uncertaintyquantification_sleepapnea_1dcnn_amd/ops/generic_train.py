"""Host orchestration of the HIP training kernels for ANY :class:`ModelSpec`.

The reference architecture trains on its own LDS-resident kernels (``ops/train_ops.py``).  Every
other architecture the spec expresses -- the opt-in ``MaxPool1D(2)`` blocks (the
north star's "Conv1D -> BN -> ReLU -> MaxPool1D -> Dropout" stack), the "30 s single-channel"
``ModelSpec(30, 1)``, other filter / kernel sizes -- trains here, with the reference's Keras
semantics (``models/cnn_baseline_train.py:55-102``: Conv1D(relu) -> BN(batch stats, moving
update) -> [pool] -> Dropout, BCE, Adam):

  per block, forward       ``gt_conv`` mode 1   z = relu(conv(h) + b) + BN moment slots (MFMA)
                           ``gt_bn_finalize``   scale / shift / mean / rstd + moving update
                           ``gt_apply``         BN + pool + dropout -> next input (zero-padded rows)
  head                     ``gt_head``: GAP + Dense + BCE + dlogit + dense grads, one launch
  weights                  ``gt_pack``: every block's forward + dgrad MFMA fragments, one launch
  per block, backward      ``gt_bwd`` stats     sum(dy), sum(dy xhat) (dropout/pool routed back)
                           ``gt_bwd_finalize``  dgamma, dbeta, BN-backward coefficients
                           ``gt_bwd`` dz        dz (zero-padded rows) + bias gradient
                           ``gt_conv`` mode 2   dgrad = conv(dz, flipped W^T) (MFMA)
                           ``gt_wgrad``         dW[tap] = Xpad[tap : tap + R]^T dZpad: split-K MFMA
                                                over the rows (csrc/generic_wgrad.hip; round 1
                                                ran it as hipBLASLt strided-batched GEMMs)
  Adam                     one multi-tensor launch over the flat buffer (``csrc/adam.hip``)

The zero-padded row layout (every sample's rows framed by k//2 zero rows, plus k//2 guard rows
at both ends) is what makes wgrad a plain GEMM: the rows of tap ``j`` are the contiguous slice
starting at row ``j`` of the padded input, so no im2col buffer is materialised.

Dropout masks are the pure function of (seed, layer, pass, window, t, channel) used everywhere
(``ops/rng.py``), keyed by the global window id, so data-parallel shards draw exactly the masks of
the single-device batch.  ``sync`` (SyncBN) all-reduces the forward moment slots and the backward
sums.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ..models.spec import ModelSpec
from . import _ext, fused, generic, rng

TRAIN_PASS_BASE = 1 << 30  # == training/step.py
SLOTS = 16  # == kStatSlots (csrc/generic_conv.hip, csrc/generic_train.hip)
DET_BWD_SLOTS = 256  # deterministic mode: workgroups (= partial slots) of each backward-sum launch
DET_WGRAD_GROUPS = 16  # deterministic mode: row groups (= partial slices) of each wgrad launch
# conv kernels of the fp32 precision path: "x3" = fp16x3 MFMA (csrc/gx3_conv.hip: 22-bit operand
# splits, fp32 accumulation, ~fp32 GEMM rounding, 3 bf16-rate MFMAs per 32-deep k-step) or "exact" =
# the fp32-input MFMA (csrc/gf32_conv.hip: exact fp32 products at 1/16 of the bf16 rate)
FP32_ENGINE = "x3"


def deterministic() -> bool:
    """The generic path follows the package-wide switch (``ops/train_ops.set_deterministic``)."""
    from . import train_ops

    return bool(train_ops.DETERMINISTIC)


def supports_fp32(spec: ModelSpec) -> bool:
    """True if the fp32 kernels (``csrc/gf32_conv.hip`` + the fp32 instantiations of the elementwise
    kernels) implement ``spec`` -- any architecture the generic path handles, the reference one included."""
    if not generic.supports(spec) or any(b.kernel_size > 15 for b in spec.blocks):
        return False
    if _ext.available():
        return True
    if not _ext.fallback_allowed():
        _ext.require()
    return False


def supports(spec: ModelSpec) -> bool:
    """True if the generic HIP training kernels implement ``spec`` (the same shapes as the generic
    inference kernels).  On a GPU box a missing extension raises unless APNEAUQ_ALLOW_FALLBACK=1."""
    if not generic.supports(spec) or any(b.kernel_size > 15 for b in spec.blocks):  # gt_wgrad: k <= 15
        return False
    if _ext.available():
        return True
    if not _ext.fallback_allowed():
        _ext.require()
    return False


class GenericTrainWorkspace:
    """Device buffers of one model for batches of up to ``batch`` windows."""

    def __init__(self, model, batch: int, with_backward: bool = True, det: Optional[bool] = None, f32: bool = False):
        spec: ModelSpec = model.spec
        dev = model.store.device
        self.model = model
        self.B = int(batch)
        self.with_backward = with_backward
        # f32: precision="fp32" -- fp32 activations / gradients; the convs on the fp16x3 MFMA
        # (csrc/gx3_conv.hip) or, with FP32_ENGINE "exact", the fp32-input MFMA (csrc/gf32_conv.hip)
        self.f32 = bool(f32)
        self.x3 = self.f32 and FP32_ENGINE == "x3"
        # deterministic mode: every cross-workgroup sum -- BN moments, backward sums, bias,
        # weight and head gradients -- goes through per-workgroup partial slots written with plain
        # stores and added in a fixed order (csrc/generic_*.hip ``det``), instead of fp32 atomics.
        # The fp32 path is always deterministic.
        self.det = True if self.f32 else (deterministic() if det is None else bool(det))
        B, bf = self.B, (torch.float32 if self.f32 else torch.bfloat16)
        self.L = spec.lengths()
        self.ch = spec.channels()
        self.ks = [b.kernel_size for b in spec.blocks]
        self.pads = [(k - 1) // 2 for k in self.ks]
        self.rs = [self.L[l] + 2 * self.pads[l] for l in range(len(spec.blocks))]
        nl = len(spec.blocks)
        # layer inputs in the zero-padded row layout: data row (n, t) at n * rs + 2 p + t
        self.xin = [torch.zeros(2 * self.pads[l] + B * self.rs[l], self.ch[l], dtype=bf, device=dev) for l in range(nl)]
        self.z = [torch.empty(B * self.L[l], self.ch[l + 1], dtype=bf, device=dev) for l in range(nl)]
        self.hlast = torch.empty(B * self.L[-1], self.ch[-1], dtype=bf, device=dev)
        # forward moment slots: (slots, 2, C); deterministic: one per (conv workgroup of 128 rows, wave row)
        fslots = [max(SLOTS, 2 * -(-B * self.L[l] // 128)) if self.det else SLOTS for l in range(nl)]
        sizes = [fslots[l] * 2 * self.ch[l + 1] for l in range(nl)]
        # + the fp16x3 operand maxima (fp32 bits as int32, atomicMax): [conv input of block l] * nl,
        # [dZ of block l] * nl -- zeroed with the moment slots every forward
        self.st_all = torch.zeros(sum(sizes) + 2 * nl, device=dev)
        self.st = list(torch.split(self.st_all[: sum(sizes)], sizes))
        amax = self.st_all[sum(sizes):].view(torch.int32)
        self.amax_x = [amax[l:l + 1] for l in range(nl)]
        self.amax_dz = [amax[nl + l:nl + l + 1] for l in range(nl)]
        self.bn = [torch.zeros(4 * self.ch[l + 1], device=dev) for l in range(nl)]
        if with_backward:
            # dz of block l, zero-padded rows (n, t) at n * rs + p + t; dh[l] = dL/d(input of block l)
            self.dzp = [torch.zeros(B * self.rs[l], self.ch[l + 1], dtype=bf, device=dev) for l in range(nl)]
            self.dh = [torch.empty(B * self.L[l], self.ch[l], dtype=bf, device=dev) if l > 0 else None
                       for l in range(nl)]
            bslots = DET_BWD_SLOTS if self.det else SLOTS
            bsizes = [bslots * 2 * self.ch[l + 1] for l in range(nl)]
            self.bst_all = torch.zeros(sum(bsizes), device=dev)
            self.bst = list(torch.split(self.bst_all, bsizes))
            # bias-gradient slots (slots, C) per block, zeroed with bst_all
            self.dbs_all = torch.zeros(sum(bsizes) // 2, device=dev)
            self.dbs = [t.view(bslots, -1) for t in torch.split(self.dbs_all, [s // 2 for s in bsizes])]
            # deterministic mode: wgrad row-group partials (shared by the sequential wgrad launches) and
            # the head's per-workgroup records
            wmax = max(self.ks[l] * self.ch[l] * self.ch[l + 1] for l in range(nl))
            if self.f32:  # gf_wgrad row groups: up to ~512 workgroups per layer (csrc/gf32_conv.hip)
                want = [-(-512 // (-(-self.ch[l] // 32) * -(-self.ch[l + 1] // 64))) for l in range(nl)]
                nf = max(w * self.ks[l] * self.ch[l] * self.ch[l + 1] for l, w in enumerate(want))
                self.wpart = torch.empty(min(nf, 1 << 24), device=dev)
            else:
                self.wpart = torch.empty(DET_WGRAD_GROUPS * wmax, device=dev) if self.det else None
            self.hpart = torch.empty(-(-B // 4) * (self.ch[-1] + 2), device=dev) if self.det else None
            self.coef = [torch.zeros(2 * self.ch[l + 1], device=dev) for l in range(nl)]
            self.y = torch.zeros(B, device=dev)
            self.prob = torch.zeros(B, device=dev)
            self.dlog = torch.zeros(B, device=dev)
            self.head_loss = torch.zeros(1, device=dev)
            # [unused, Adam iterations]: the eager step computes Adam's bias correction on the device from
            # this counter, exactly as the captured step does (eager == graph arithmetic)
            self.counters = torch.zeros(2, dtype=torch.int32, device=dev)
            store = model.store
            self.grad = torch.zeros_like(store.flat)
            self.gviews = {}
            for n in store.trainable:
                off = store.offsets[n]
                self.gviews[n] = self.grad[off: off + store.views[n].numel()].view(store.shapes[n])

    def load_input(self, x: torch.Tensor) -> None:
        n, p = x.shape[0], self.pads[0]
        self.xin[0][p: p + n * self.rs[0]].view(n, self.rs[0], self.ch[0])[:, p: p + self.L[0]].copy_(x)

    def pack(self, backward: bool):
        """MFMA fragments of every conv kernel (forward; + dgrad orientation when training), all blocks
        in one HIP launch into buffers allocated once (the weights change every step): bf16, or on the
        fp32 path the fp16x3 hi/lo fragments with one power-of-two prescale per kernel (two launches,
        ``gx3_pack``; the scales in ``self.wsc``).  The exact-fp32 kernels read the Keras kernels in place."""
        v = self.model.store.views
        nl = len(self.ks)
        w = [v[f"conv1d_{l + 1}/kernel"] for l in range(nl)]
        if self.f32 and not self.x3:
            return w, w
        if self.x3:
            # inference packs once per parameter version (training repacks every step)
            key = (id(self.model.store), self.model.store.version, bool(backward))
            if not backward and getattr(self, "_xpack_key", None) == key:
                return self._xf, [None] * nl
            self._xpack_key = key
            if getattr(self, "_xf", None) is None:
                dev = self.model.store.device
                self._xf, self._xd = [], []
                for l in range(nl):
                    k, cin, cout = self.ks[l], self.ch[l], self.ch[l + 1]
                    self._xf.append(torch.empty(2 * ((k * cin + 31) // 32) * 512 * ((cout + 15) // 16),
                                                dtype=torch.float16, device=dev))
                    self._xd.append(torch.empty(2 * ((k * cout + 31) // 32) * 512 * ((cin + 15) // 16),
                                                dtype=torch.float16, device=dev) if l > 0 else
                                    torch.empty(0, dtype=torch.float16, device=dev))
                self._xnone = torch.empty(0, dtype=torch.float16, device=dev)
                self._wsc_all = torch.ones(4 * nl, device=dev)  # one 16-B aligned slot per block
                self.wsc = [self._wsc_all[4 * l:4 * l + 1] for l in range(nl)]
                self._wmaxpart = torch.empty(16 * nl, device=dev)
            dgr = self._xd if backward else [self._xnone] * nl
            _ext.ops().gx3_pack(w, self._xf, dgr, self.wsc, list(self.ks), list(self.ch[:-1]), list(self.ch[1:]),
                                self._wmaxpart)
            return self._xf, [d if d.numel() else None for d in dgr]
        if getattr(self, "_wf", None) is None:
            dev = self.model.store.device
            self._wf, self._wd = [], []
            for l in range(nl):
                k, cin, cout = self.ks[l], self.ch[l], self.ch[l + 1]
                nf = ((k * cin + 31) // 32, (cout + 15) // 16, 64, 8)
                nd = ((k * cout + 31) // 32, (cin + 15) // 16, 64, 8)
                self._wf.append(torch.empty(nf, dtype=torch.bfloat16, device=dev))
                self._wd.append(torch.empty(nd, dtype=torch.bfloat16, device=dev) if l > 0 else
                                torch.empty(0, dtype=torch.bfloat16, device=dev))
            self._none = torch.empty(0, dtype=torch.bfloat16, device=dev)
        w = [v[f"conv1d_{l + 1}/kernel"] for l in range(nl)]
        dgr = self._wd if backward else [self._none] * nl
        _ext.ops().gt_pack(w, self._wf, dgr, list(self.ks), list(self.ch[:-1]), list(self.ch[1:]))
        return self._wf, [d if d.numel() else None for d in dgr]


def _frag(w: torch.Tensor) -> torch.Tensor:
    cout = w.shape[2]
    cpad = (cout + 15) // 16 * 16
    return fused.pack_conv_fragments(torch.nn.functional.pad(w, (0, cpad - cout)))


def _get_ws(model, batch: int, with_backward: bool = True, f32: bool = False) -> GenericTrainWorkspace:
    attr = ("_gtrain_ws" if with_backward else "_gfwd_ws") + ("32" if f32 else "")
    ws = getattr(model, attr, None)
    if (ws is None or ws.B < batch or (not f32 and ws.det != deterministic())
            or (f32 and ws.x3 != (FP32_ENGINE == "x3"))):
        ws = GenericTrainWorkspace(model, batch, with_backward=with_backward, f32=f32)
        setattr(model, attr, ws)
    return ws


def _forward(ws: GenericTrainWorkspace, n: int, global_n: int, seed: int, pass_id: int, window_offset: int,
             dropout: bool, update_moving: bool, sync: Optional[Callable], wf, keys_dev=None,
             zero_stats: bool = True) -> torch.Tensor:
    """Batch-statistics forward of ``n`` windows already loaded in ``ws.xin[0]``; returns the
    last block's output (n, L_out, C) bf16.  ``keys_dev`` (int32 (blocks,)) makes the kernels read
    the dropout stream keys from device memory (HIP-graph replays).  ``zero_stats=False``: the caller
    has zeroed ``ws.st_all`` already (one launch with its other accumulators)."""
    o = _ext.ops()
    spec, v = ws.model.spec, ws.model.store.views
    nl = len(spec.blocks)
    if zero_stats:
        ws.st_all.zero_()
    ws._running_key = None  # ws.bn gets the batch affine below (running_affine must rebuild it)
    for l, b in enumerate(spec.blocks):
        i = l + 1
        cin, cout, L = ws.ch[l], ws.ch[l + 1], ws.L[l]
        if ws.x3:
            o.gx3_conv(ws.xin[l], wf[l], ws.wsc[l], v[f"conv1d_{i}/bias"], ws.z[l], ws.st[l], ws.amax_x[l], n, L, cin,
                       cout, ws.ks[l], 1, ws.rs[l], 2 * ws.pads[l], ws.det)
        else:
            conv = o.gf_conv if ws.f32 else o.gt_conv
            conv(ws.xin[l], wf[l], v[f"conv1d_{i}/bias"], ws.z[l], ws.st[l], n, L, cin, cout, ws.ks[l], 1,
                 ws.rs[l], 2 * ws.pads[l], ws.det)
        if sync is not None:
            sync(ws.st[l])
        # consumes ws.st[l]: a large slot table (deterministic mode) is summed in place, its first slots
        # overwritten by packed fp64 range sums (csrc/generic_train.hip slot_partial_kernel), so nothing
        # may read ws.st[l] after this call
        o.gt_bn_finalize(ws.st[l], cout, 1.0 / (global_n * L), v[f"batchnorm_{i}/gamma"], v[f"batchnorm_{i}/beta"],
                         spec.bn_epsilon, spec.bn_momentum, v[f"batchnorm_{i}/moving_mean"],
                         v[f"batchnorm_{i}/moving_variance"], bool(update_moving), ws.bn[l])
        if l + 1 < nl:
            out, out_rs, out_off = ws.xin[l + 1], ws.rs[l + 1], 2 * ws.pads[l + 1]
        else:
            out, out_rs, out_off = ws.hlast, ws.L[-1], 0
        drop = bool(dropout and b.dropout > 0)
        o.gt_apply(ws.z[l], ws.bn[l], out, n, L, cout, bool(b.pool), out_rs, out_off, drop,
                   rng.dropout_threshold(b.dropout), _inv_keep(b.dropout), rng.stream_key(seed, l, pass_id),
                   int(window_offset), None if keys_dev is None else keys_dev[l:l + 1])
    return ws.hlast[: n * ws.L[-1]].view(n, ws.L[-1], ws.ch[-1])


def _inv_keep(rate: float) -> float:
    return 1.0 / (1.0 - rate) if rate < 1.0 else 0.0


def _grads(model, ws: GenericTrainWorkspace, y: torch.Tensor, n: int, gb: int, pass_id: int, window_offset: int,
           sync: Optional[Callable], keys_dev=None):
    """Forward + head + backward of the ``n`` windows in ``ws.xin[0]`` into ``ws.grad`` (zeroed here).
    Every launch is a HIP kernel of this package (no library GEMM, no host sync): capturable."""
    spec: ModelSpec = model.spec
    o = _ext.ops()
    v, g = model.store.views, ws.gviews
    nl = len(spec.blocks)
    seed = model.seed
    wf, wd = ws.pack(backward=True)
    # every accumulator of the step (forward / backward BN moments, bias slots, gradient, loss): one launch
    o.zero_buffers([ws.st_all, ws.bst_all, ws.dbs_all, ws.grad, ws.head_loss])
    h = _forward(ws, n, gb, seed, pass_id, window_offset, True, True, sync, wf, keys_dev, zero_stats=False)
    # head: GAP + Dense + BCE(logits) + dlogit + dense gradients (mean over the global batch), one launch
    wdense = v["output_layer/kernel"].reshape(-1)
    ws.y[:n].copy_(y.reshape(-1))
    o.gt_head(h, wdense, v["output_layer/bias"], ws.y, ws.prob, ws.dlog, ws.head_loss, g["output_layer/kernel"],
              g["output_layer/bias"], n, ws.L[-1], ws.ch[-1], 1.0 / gb, ws.hpart)
    dlog = ws.dlog
    for l in range(nl - 1, -1, -1):
        i, b = l + 1, spec.blocks[l]
        cin, cout, L, p, k = ws.ch[l], ws.ch[l + 1], ws.L[l], ws.pads[l], ws.ks[l]
        drop = b.dropout > 0
        thr, ik, skey = rng.dropout_threshold(b.dropout), _inv_keep(b.dropout), rng.stream_key(seed, l, pass_id)
        kd = None if keys_dev is None else keys_dev[l:l + 1]
        if l == nl - 1:
            up = dict(dh=None, dlog=dlog, w=wdense, invL=1.0 / ws.L[-1])
        else:
            up = dict(dh=ws.dh[l + 1], dlog=None, w=None, invL=1.0)
        o.gt_bwd(False, ws.z[l], ws.bn[l], up["dh"], up["dlog"], up["w"], up["invL"], n, L, cout, bool(b.pool), drop,
                 thr, ik, skey, int(window_offset), ws.bst[l], None, None, None, 0, 0, None, kd, ws.det)
        if sync is not None:
            sync(ws.bst[l])
        # + the bias gradient of block l + 1 (its slots are complete) as extra workgroups of the finalize
        above = (ws.dbs[l + 1], g[f"conv1d_{i + 1}/bias"]) if l + 1 < nl else (None, None)
        o.gt_bwd_finalize(ws.bst[l], cout, 1.0 / (gb * L), ws.coef[l], g[f"batchnorm_{i}/gamma"],
                          g[f"batchnorm_{i}/beta"], *above)
        o.gt_bwd(True, ws.z[l], ws.bn[l], up["dh"], up["dlog"], up["w"], up["invL"], n, L, cout, bool(b.pool), drop,
                 thr, ik, skey, int(window_offset), None, ws.coef[l], v[f"batchnorm_{i}/gamma"], ws.dzp[l], ws.rs[l], p,
                 ws.dbs[l], kd, ws.det)
        if l == 0:  # block 1's bias gradient: a finalize launch with no BN part
            o.gt_bwd_finalize(ws.bst[0], 0, 1.0, ws.coef[0], g["batchnorm_1/gamma"], g["batchnorm_1/beta"], ws.dbs[0],
                              g["conv1d_1/bias"])
        if ws.x3:
            # dgrad publishes dZ's tensor maximum for the wgrad prescale (block 1: no dgrad, amax kernel)
            if l > 0:
                o.gx3_conv(ws.dzp[l], wd[l], ws.wsc[l], None, ws.dh[l], None, ws.amax_dz[l], n, L, cout, cin, k, 2,
                           ws.rs[l], p)
            else:
                o.gx3_amax(ws.dzp[l], n * ws.rs[l] * cout, ws.amax_dz[l])
            o.gx3_wgrad(ws.xin[l], ws.dzp[l], ws.amax_x[l], ws.amax_dz[l], n * ws.rs[l], cin, cout, k,
                        g[f"conv1d_{i}/kernel"], ws.wpart)
            continue
        if l > 0:
            (o.gf_conv if ws.f32 else o.gt_conv)(ws.dzp[l], wd[l], None, ws.dh[l], None, n, L, cout, cin, k, 2,
                                                 ws.rs[l], p)
        # wgrad: dW[tap] = Xpad[tap : tap + R]^T dZpad (R = n * rs rows), split-K MFMA into the zeroed grad
        if ws.f32:
            o.gf_wgrad(ws.xin[l], ws.dzp[l], n * ws.rs[l], cin, cout, k, g[f"conv1d_{i}/kernel"], ws.wpart)
        else:
            o.gt_wgrad(ws.xin[l], ws.dzp[l], n * ws.rs[l], cin, cout, k, g[f"conv1d_{i}/kernel"], ws.wpart)


def _f32(model) -> bool:
    return getattr(model, "train_precision", "bf16") == "fp32"


def train_step(model, x: torch.Tensor, y: torch.Tensor, grad_allreduce=None, sync: Optional[Callable] = None,
               global_batch: Optional[int] = None, window_offset: int = 0, sync_world: int = 1):
    """One Keras-semantics optimizer step on the generic HIP kernels (bf16, or fp32 when the model's
    ``train_precision`` is "fp32"); returns (loss_sum, probs)."""
    n = int(x.shape[0])
    gb = int(global_batch or n)
    ws = _get_ws(model, n, f32=_f32(model))
    ws.load_input(x)
    _grads(model, ws, y, n, gb, TRAIN_PASS_BASE + model._train_step_counter, window_offset, sync)
    g = ws.gviews
    if sync is not None and sync_world > 1:  # the synced sums made dgamma / dbeta global already
        for i in range(1, len(model.spec.blocks) + 1):
            g[f"batchnorm_{i}/gamma"].div_(sync_world)
            g[f"batchnorm_{i}/beta"].div_(sync_world)
    scale = 1.0
    if grad_allreduce is not None:
        scale = grad_allreduce(ws.grad)
    model.optimizer.step(model.store.flat, ws.grad, grad_scale=scale, counters=ws.counters)
    return ws.head_loss.double().sum(), ws.prob[:n]


class GraphedGenericStep:
    """The whole generic-spec training step of one batch size captured once as a HIP graph.

    Per step the generic path issues ~9 launches per block (conv, BN finalize, apply, two backward
    passes, finalize, bias sum, dgrad, wgrad) plus head, packing and Adam: ~60 launches for six
    blocks, ~1 ms of host dispatch at batch 1024.  Everything a step varies comes from device counters
    ``[dropout step, Adam iterations]`` bumped by the graph's last node: its first node derives the
    dropout stream keys from the step counter (``stream_keys``) and Adam's bias correction reads the
    iteration counter, so a replay reads no host-written memory and is exactly the eager step.  The
    host mirrors the counters and re-syncs them only when they were changed outside (an eager step,
    a restore).  Single device only (data-parallel steps all-reduce through torch.distributed)."""

    def __init__(self, model, batch: int):
        self.model = model
        self.batch = int(batch)
        dev = model.store.device
        spec = model.spec
        self.f32 = _f32(model)
        self.ws = GenericTrainWorkspace(model, self.batch, f32=self.f32)
        self.det = self.ws.det
        self.x_in = torch.zeros(self.batch, spec.input_length, spec.input_channels, device=dev)
        self.y_in = torch.zeros(self.batch, device=dev)
        self.keys = torch.zeros(len(spec.blocks), dtype=torch.int32, device=dev)
        self.counters = torch.zeros(2, dtype=torch.int32, device=dev)  # [dropout step, Adam iterations]
        model.optimizer._ensure(model.store.flat)
        from . import train_ops

        self.bound = train_ops.bound_key(model)
        self._sync_counters()
        self.ws.pack(backward=True)  # allocates the fragment buffers outside the capture (no model change)
        from .train_ops import capture_graph

        self.graph = capture_graph(self._body, dev)

    def _state(self):
        return (int(self.model._train_step_counter), int(self.model.optimizer.iterations))

    def _sync_counters(self):
        st = self._state()
        self.counters.copy_(torch.tensor(st, dtype=torch.int32))
        self._dev_state = st

    def _body(self):
        ws, n, m = self.ws, self.batch, self.model
        seed = int(m.seed) & ((1 << 64) - 1)
        _ext.ops().stream_keys(self.keys, self.counters, seed - (1 << 64) if seed >= (1 << 63) else seed,
                               TRAIN_PASS_BASE)
        ws.load_input(self.x_in)
        _grads(m, ws, self.y_in, n, n, TRAIN_PASS_BASE, 0, None, keys_dev=self.keys)
        opt = m.optimizer
        _ext.ops().adam_step(m.store.flat, ws.grad, opt.m, opt.v, opt.beta_1, opt.beta_2, opt.learning_rate,
                             opt.epsilon, 1.0, self.counters)
        _ext.ops().bump_counters(self.counters)

    def __call__(self, x: torch.Tensor, y: torch.Tensor):
        m = self.model
        if self._state() != self._dev_state:
            self._sync_counters()
        self.x_in.copy_(x)
        self.y_in.copy_(y.reshape(-1))
        self.graph.replay()
        m.optimizer.iterations += 1
        self._dev_state = (self._dev_state[0] + 1, self._dev_state[1] + 1)
        return self.ws.head_loss.double().sum(), self.ws.prob[: self.batch]


def graph_train_step(model, x: torch.Tensor, y: torch.Tensor):
    """Replay (capturing on first use) the graphed generic step for this batch size."""
    from . import train_ops

    g = getattr(model, "_gtrain_graphs", None)
    if g is None:
        g = model._gtrain_graphs = {}
    n = int(x.shape[0])
    cur = g.get(n)
    if (cur is None or not train_ops._same_bound(cur.bound, train_ops.bound_key(model)) or cur.f32 != _f32(model)
            or (not cur.f32 and cur.det != deterministic()) or (cur.f32 and cur.ws.x3 != (FP32_ENGINE == "x3"))):
        g[n] = cur = GraphedGenericStep(model, n)
    return cur(x, y)


@torch.no_grad()
def forward_batch_stats(model, x: torch.Tensor, n_pass: int, pass_base: int, seed: int, update_moving: bool = True,
                        sync: Optional[Callable] = None, window_offset: int = 0,
                        global_n: Optional[int] = None, f32: Optional[bool] = None) -> torch.Tensor:
    """MC Dropout with BN on per-pass batch statistics of the whole set (the reference's
    ``model(x, training=True)``) for any spec: (T, N) probabilities, one layer-synchronous
    sweep per pass.  ``f32`` (default: the model's inference ``precision`` is "fp32"): fp32 activations
    and fp32-input MFMA convs (exact fp32 products, the reference's precision); else bf16."""
    n = int(x.shape[0])
    gn = int(global_n or n)
    if f32 is None:
        f32 = getattr(model, "precision", "fp32") == "fp32"
    ws = _get_ws(model, n, with_backward=False, f32=bool(f32))
    ws.load_input(x)
    wf, _ = ws.pack(backward=False)
    v = model.store.views
    wdense = v["output_layer/kernel"].reshape(-1)
    out = torch.empty(n_pass, n, device=x.device)
    for t in range(n_pass):
        h = _forward(ws, n, gn, seed, pass_base + t, window_offset, True, update_moving, sync, wf)
        out[t] = torch.sigmoid(torch.addmv(v["output_layer/bias"], h.float().mean(dim=1), wdense))
    model.store.bump()
    return out


def running_affine(model, ws: GenericTrainWorkspace) -> None:
    """BN on the moving statistics, as the (4, C) rows [scale, shift, mean, rstd] gt_apply reads
    (recomputed only when the store's parameters changed since the last call on this workspace)."""
    spec, v = model.spec, model.store.views
    key = (id(model.store), model.store.version)
    if getattr(ws, "_running_key", None) == key:
        return
    ws._running_key = key
    for l in range(len(spec.blocks)):
        i = l + 1
        mm, mv = v[f"batchnorm_{i}/moving_mean"], v[f"batchnorm_{i}/moving_variance"]
        rstd = torch.rsqrt(mv + spec.bn_epsilon)
        scale = v[f"batchnorm_{i}/gamma"] * rstd
        ws.bn[l].copy_(torch.cat([scale, v[f"batchnorm_{i}/beta"] - mm * scale, mm, rstd]))


# fp32 inference workspace cap (activations of one window chunk, all layers): large Deep-Ensemble /
# MC-Dropout sets are processed in window chunks that fit it, so the cached workspace stays bounded
F32_INFER_WS_BYTES = 1 << 31


def _f32_chunk_windows(model) -> int:
    spec = model.spec
    L, ch = spec.lengths(), spec.channels()
    per = sum((L[l] + b.kernel_size) * ch[l] + L[l] * ch[l + 1] for l, b in enumerate(spec.blocks)) * 4
    return max(1, F32_INFER_WS_BYTES // per)


@torch.no_grad()
def forward_running_f32(model, x: torch.Tensor, n_pass: int = 1, dropout: bool = False, seed: int = 0,
                        pass_offset: int = 0, window_offset: int = 0, logits: bool = False) -> torch.Tensor:
    """Inference with BN on the moving statistics (Deep-Ensemble ``predict`` / standard MC Dropout,
    ``uq_techniques.py:22-30``) at the reference's fp32 for ANY spec -- the MaxPool1D variant of the
    thesis' ``ensemble_cnn`` members (``evaluate_de_global.py:18-38``), the 30 s single-channel window --
    on the fp16x3 conv (``csrc/gx3_conv.hip``; FP32_ENGINE "exact": ``csrc/gf32_conv.hip``) and the fp32
    BN / pool / dropout kernels:
    (n_pass, N) probabilities (or logits).  The passes run one after the other (each its own dropout
    stream, keyed by the global window id); windows in chunks of at most ``F32_INFER_WS_BYTES`` of
    activations (the dropout keys stay global: chunk s starts at window_offset + s)."""
    n = int(x.shape[0])
    out = torch.empty(n_pass, n, dtype=torch.float32, device=x.device)
    if n == 0:
        return out
    step = _f32_chunk_windows(model)
    for s in range(0, n, step):
        e = min(n, s + step)
        out[:, s:e] = _forward_running_f32_chunk(model, x[s:e], n_pass, dropout, seed, pass_offset,
                                                 window_offset + s, logits)
    return out


def _forward_running_f32_chunk(model, x, n_pass, dropout, seed, pass_offset, window_offset, logits):
    n = int(x.shape[0])
    out = torch.empty(n_pass, n, dtype=torch.float32, device=x.device)
    spec, o = model.spec, _ext.ops()
    ws = _get_ws(model, n, with_backward=False, f32=True)
    running_affine(model, ws)
    ws.load_input(x)
    wf, _ = ws.pack(backward=False)
    v = model.store.views
    wdense = v["output_layer/kernel"].reshape(-1)
    nl = len(spec.blocks)
    conv0 = True
    for t in range(n_pass if dropout else 1):
        for l, b in enumerate(spec.blocks):
            i = l + 1
            cin, cout, L = ws.ch[l], ws.ch[l + 1], ws.L[l]
            if l > 0 or conv0:  # block 1 does not depend on the pass (no dropout before it)
                if ws.x3:
                    o.gx3_conv(ws.xin[l], wf[l], ws.wsc[l], v[f"conv1d_{i}/bias"], ws.z[l], ws.st[l], None, n, L,
                               cin, cout, ws.ks[l], 1, ws.rs[l], 2 * ws.pads[l], True)
                else:
                    o.gf_conv(ws.xin[l], wf[l], v[f"conv1d_{i}/bias"], ws.z[l], ws.st[l], n, L, cin, cout,
                              ws.ks[l], 1, ws.rs[l], 2 * ws.pads[l], True)
            if l + 1 < nl:
                dst, drs, doff = ws.xin[l + 1], ws.rs[l + 1], 2 * ws.pads[l + 1]
            else:
                dst, drs, doff = ws.hlast, ws.L[-1], 0
            drop = bool(dropout and b.dropout > 0)
            o.gt_apply(ws.z[l], ws.bn[l], dst, n, L, cout, bool(b.pool), drs, doff, drop,
                       rng.dropout_threshold(b.dropout), _inv_keep(b.dropout),
                       rng.stream_key(seed, l, pass_offset + t), int(window_offset), None)
        conv0 = False
        h = ws.hlast[: n * ws.L[-1]].view(n, ws.L[-1], ws.ch[-1])
        lg = torch.addmv(v["output_layer/bias"], h.mean(dim=1), wdense)
        out[t] = lg if logits else torch.sigmoid(lg)
    if not dropout:
        out[1:] = out[0]
    return out
