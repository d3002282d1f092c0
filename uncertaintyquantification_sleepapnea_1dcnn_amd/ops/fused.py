"""Host side of the fused whole-network inference kernel (``csrc/fused_forward.hip``).

``pack_blob`` turns one model's Keras-ordered parameters into the byte layout the kernel reads:
per block the conv kernel transposed to ``W^T[co][k]`` (``k = tap*Cin + ci``, zero-padded to a
multiple of 32) and re-ordered into v_mfma_f32_16x16x32_bf16 A-operand fragments (1 KiB per
(k-step, 16-channel tile), lane ``l`` holding ``co = 16*tile + (l & 15)``,
``k = 32*step + 8*(l >> 4) + j``), then the fp32 epilogue vectors ``[bias | bn_scale | bn_shift]``
(inference BatchNorm folded to an affine), then the dense head.  The offsets are computed here
and cross-checked against the kernel's own ``fused_layout()``.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import torch

from ..models.spec import DEFAULT_SPEC, ModelSpec
from . import _ext, rng

FUSED_CHANNELS = (4, 128, 192, 224, 96, 256, 96)
FUSED_KSIZES = (7, 5, 3, 7, 9, 9)
FUSED_LENGTH = 60


def supports(spec: ModelSpec) -> bool:
    """True if the fused kernel implements this architecture (the reference's no-pool CNN)."""
    return (spec.input_length == FUSED_LENGTH and tuple(spec.channels()) == FUSED_CHANNELS
            and tuple(b.kernel_size for b in spec.blocks) == FUSED_KSIZES and not spec.has_pool)


POOLED_PATTERN = (True, True, True, True, True, False)


def pooled_supported(spec: ModelSpec) -> bool:
    """True if ``csrc/fused_tiled.hip`` (PooledNet) implements this architecture: the reference CNN
    with MaxPool1D(2) after blocks 1-5 (the pooling lines of train_deep_ensemble_cnns.py:36-66)."""
    return (spec.input_length == FUSED_LENGTH and tuple(spec.channels()) == FUSED_CHANNELS
            and tuple(b.kernel_size for b in spec.blocks) == FUSED_KSIZES
            and tuple(bool(b.pool) for b in spec.blocks) == POOLED_PATTERN)


def single30_supported(spec: ModelSpec) -> bool:
    """True if ``csrc/fused_tiled.hip`` (Single30Net) implements this architecture: the reference
    filters / kernel sizes on the north star's 30 s single-channel window, no pooling."""
    return (spec.input_length == 30 and tuple(spec.channels()) == (1,) + FUSED_CHANNELS[1:]
            and tuple(b.kernel_size for b in spec.blocks) == FUSED_KSIZES and not spec.has_pool)


def tiled_net(spec: ModelSpec) -> Optional[int]:
    """Net id of ``csrc/fused_tiled.hip`` for this spec (0 pooled, 1 single-channel 30 s), else None."""
    return 0 if pooled_supported(spec) else 1 if single30_supported(spec) else None


_WARNED = set()


def warn_unsupported(spec: ModelSpec, what: str) -> None:
    """One warning per (architecture, path) that runs on the fp32 PyTorch path instead of HIP."""
    key = (repr(spec), what)
    if key not in _WARNED and torch.cuda.is_available():
        _WARNED.add(key)
        import warnings

        warnings.warn(f"apneauq: no HIP {what} kernel for this architecture (input {spec.input_length}x"
                      f"{spec.input_channels}, pool={spec.has_pool}); using the fp32 PyTorch path", stacklevel=3)


EPI_ROWS = 8  # per-channel epilogue constants [s, t', lo, hi] as-is, then pre-scaled by 1/(1-rate)


def epilogue_constants(bias: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor) -> torch.Tensor:
    """Fold bias + ReLU + BN affine into one fma + one clamp (``v_fma`` + ``v_med3``):

    ``relu(acc + b) * s + t == clamp(acc * s + (b * s + t), lo, hi)`` with ``[lo, hi] = [t, +inf]``
    for ``s >= 0`` and ``[-inf, t]`` for ``s < 0``.  Returns (4, C) fp32 rows [s, t', lo, hi]."""
    s = scale.float()
    t = shift.float()
    inf = torch.full_like(t, float("inf"))
    lo = torch.where(s >= 0, t, -inf)
    hi = torch.where(s >= 0, inf, t)
    return torch.stack([s, bias.float() * s + t, lo, hi])


def _ceil(a: int, b: int) -> int:
    return (a + b - 1) // b * b


def layout() -> Dict[str, object]:
    ch, ks = FUSED_CHANNELS, FUSED_KSIZES
    woff, eoff = [], []
    off = 0
    for l in range(6):
        woff.append(off)
        off += ((ch[l] * ks[l] + 31) // 32) * (ch[l + 1] // 16) * 1024
    for l in range(6):
        eoff.append(off)
        off += _ceil(EPI_ROWS * ch[l + 1] * 4, 16)
    dense = off
    total = dense + _ceil((ch[6] + 1) * 4, 16)
    return {"woff": woff, "eoff": eoff, "dense": dense, "bytes": total}


def check_layout() -> None:
    lay = layout()
    v = list(_ext.ops().fused_layout())
    want = lay["woff"] + lay["eoff"] + [lay["dense"], lay["bytes"]]
    if v[:14] != want:
        raise RuntimeError(f"fused blob layout mismatch host={want} kernel={v[:14]}")


def pack_conv_fragments(kernel: torch.Tensor) -> torch.Tensor:
    """Keras conv kernel (k, Cin, Cout) -> bf16 fragments (nstep, Cout/16, 64 lanes, 8)."""
    k, cin, cout = kernel.shape
    K = k * cin
    nstep = (K + 31) // 32
    wt = kernel.detach().float().reshape(K, cout).t()  # (cout, K), k = tap*cin + ci
    wt = torch.nn.functional.pad(wt, (0, nstep * 32 - K))
    fr = wt.reshape(cout // 16, 16, nstep, 4, 8).permute(2, 0, 3, 1, 4)  # (step, ct, h, m, j)
    return fr.reshape(nstep, cout // 16, 64, 8).to(torch.bfloat16).contiguous()


def unpack_conv_fragments(fr: torch.Tensor, k: int, cin: int, cout: int) -> torch.Tensor:
    """Inverse of :func:`pack_conv_fragments` (returns fp32 (k, Cin, Cout))."""
    nstep = fr.shape[0]
    wt = fr.float().reshape(nstep, cout // 16, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(cout, nstep * 32)
    return wt[:, : k * cin].t().reshape(k, cin, cout)


def bn_affine(spec: ModelSpec, p, i: int):
    gamma, beta = p[f"batchnorm_{i}/gamma"].float(), p[f"batchnorm_{i}/beta"].float()
    mm, mv = p[f"batchnorm_{i}/moving_mean"].float(), p[f"batchnorm_{i}/moving_variance"].float()
    scale = gamma * torch.rsqrt(mv + spec.bn_epsilon)
    return scale, beta - mm * scale


def pack_blob(spec: ModelSpec, p, bn_override: Optional[Sequence] = None) -> torch.Tensor:
    """Pack one model into the fused kernel's byte blob (uint8, on the params' device).

    ``bn_override``: optional list of 6 (scale, shift) pairs replacing the running-stat BN affine
    (used by the batch-statistics MC-Dropout parity mode).
    """
    if not (supports(spec) or tiled_net(spec) is not None):
        raise ValueError("fused kernels support only the reference filters / kernel sizes on a (60, 4) window "
                         "(without pooling or with MaxPool1D(2) after blocks 1-5) or a (30, 1) window")
    lay = layout()
    dev = p["conv1d_1/kernel"].device
    blob = torch.zeros(lay["bytes"], dtype=torch.uint8, device=dev)
    for l in range(6):
        i = l + 1
        fr = pack_conv_fragments(p[f"conv1d_{i}/kernel"].to(dev))
        b = fr.view(torch.uint8).reshape(-1)
        blob[lay["woff"][l]: lay["woff"][l] + b.numel()] = b
        if bn_override is not None:
            scale, shift = bn_override[l]
        else:
            scale, shift = bn_affine(spec, p, i)
        epi = epilogue_constants(p[f"conv1d_{i}/bias"].float().to(dev), scale.float().to(dev), shift.float().to(dev))
        rate = spec.blocks[l].dropout
        epi = torch.cat([epi, epi * (1.0 / (1.0 - rate) if rate < 1.0 else 0.0)])  # MC-Dropout rows
        e = epi.contiguous().view(torch.uint8).reshape(-1)
        blob[lay["eoff"][l]: lay["eoff"][l] + e.numel()] = e
    head = torch.cat([p["output_layer/kernel"].float().reshape(-1), p["output_layer/bias"].float().reshape(-1)]).to(dev)
    h = head.contiguous().view(torch.uint8)
    blob[lay["dense"]: lay["dense"] + h.numel()] = h
    return blob


# ------------------------------------------------------------------------------------------------
# fp16x3 blob of the fp32-faithful fused kernel (csrc/fused_tiled_x3.hip): per (k-step, channel tile)
# the hi and the lo fp16 fragment of W 2^sw (sw: one power of two per layer putting max |W| 2^sw in
# [2^13, 2^14)), then the epilogue rows with the BN scale x 2^-sw, then the dense head.
# ------------------------------------------------------------------------------------------------
def layout_x3() -> Dict[str, object]:
    ch, ks = FUSED_CHANNELS, FUSED_KSIZES
    woff, eoff = [], []
    off = 0
    for l in range(6):
        woff.append(off)
        off += 2 * ((ch[l] * ks[l] + 31) // 32) * (ch[l + 1] // 16) * 1024
    for l in range(6):
        eoff.append(off)
        off += _ceil(EPI_ROWS * ch[l + 1] * 4, 16)
    dense = off
    total = dense + _ceil((ch[6] + 1) * 4, 16)
    return {"woff": woff, "eoff": eoff, "dense": dense, "bytes": total}


def check_layout_x3() -> None:
    lay = layout_x3()
    v = list(_ext.ops().fused_layout_x3())
    want = lay["woff"] + lay["eoff"] + [lay["dense"], lay["bytes"]]
    if v[:14] != want:
        raise RuntimeError(f"fused x3 blob layout mismatch host={want} kernel={v[:14]}")


def pow2_exponent(maxabs: float) -> int:
    """The power of two that puts a nonzero ``maxabs`` into [2^13, 2^14) (0 for zero / non-finite)."""
    import math

    if not (maxabs > 0.0 and math.isfinite(maxabs)):
        return 0
    return max(-100, min(100, 14 - math.frexp(maxabs)[1]))


def pack_conv_fragments_x3(kernel: torch.Tensor):
    """Keras conv kernel (k, Cin, Cout) -> (fragments (nstep, Cout/16, 2, 64, 8) fp16 [hi, lo] of
    W 2^sw, sw)."""
    k, cin, cout = kernel.shape
    K = k * cin
    nstep = (K + 31) // 32
    w = kernel.detach().float()
    sw = pow2_exponent(float(w.abs().max()))
    wt = torch.ldexp(w.reshape(K, cout).t(), torch.tensor(float(sw), device=w.device))
    wt = torch.nn.functional.pad(wt, (0, nstep * 32 - K))
    fr = wt.reshape(cout // 16, 16, nstep, 4, 8).permute(2, 0, 3, 1, 4).reshape(nstep, cout // 16, 64, 8)
    hi = fr.to(torch.float16)
    lo = (fr - hi.float()).to(torch.float16)
    return torch.stack([hi, lo], dim=2).contiguous(), sw


def unpack_conv_fragments_x3(fr: torch.Tensor, sw: int, k: int, cin: int, cout: int) -> torch.Tensor:
    """Inverse of :func:`pack_conv_fragments_x3` (fp32 (k, Cin, Cout), hi + lo scaled back)."""
    nstep = fr.shape[0]
    w = fr[:, :, 0].float() + fr[:, :, 1].float()
    wt = w.reshape(nstep, cout // 16, 4, 16, 8).permute(1, 3, 0, 2, 4).reshape(cout, nstep * 32)
    return torch.ldexp(wt[:, : k * cin].t(), torch.tensor(float(-sw))).reshape(k, cin, cout)


def pack_blob_x3(spec: ModelSpec, p) -> torch.Tensor:
    """Pack one model into the fp16x3 fused kernel's blob (uint8, on the params' device); BN on the
    moving statistics."""
    if tiled_net(spec) is None:
        raise ValueError("the fp32 fused kernel supports the pooled (60, 4) and the single-channel (30, 1) CNN")
    lay = layout_x3()
    dev = p["conv1d_1/kernel"].device
    blob = torch.zeros(lay["bytes"], dtype=torch.uint8, device=dev)
    for l in range(6):
        i = l + 1
        fr, sw = pack_conv_fragments_x3(p[f"conv1d_{i}/kernel"].to(dev))
        b = fr.view(torch.uint8).reshape(-1)
        blob[lay["woff"][l]: lay["woff"][l] + b.numel()] = b
        scale, shift = bn_affine(spec, p, i)
        epi = epilogue_constants(p[f"conv1d_{i}/bias"].float().to(dev), scale.float().to(dev), shift.float().to(dev))
        epi[0] = torch.ldexp(epi[0], torch.tensor(float(-sw), device=dev))  # undo the weight prescale
        rate = spec.blocks[l].dropout
        epi = torch.cat([epi, epi * (1.0 / (1.0 - rate) if rate < 1.0 else 0.0)])
        e = epi.contiguous().view(torch.uint8).reshape(-1)
        blob[lay["eoff"][l]: lay["eoff"][l] + e.numel()] = e
    head = torch.cat([p["output_layer/kernel"].float().reshape(-1), p["output_layer/bias"].float().reshape(-1)]).to(dev)
    h = head.contiguous().view(torch.uint8)
    blob[lay["dense"]: lay["dense"] + h.numel()] = h
    return blob


def tiled_x3_forward(x: torch.Tensor, blobs: torch.Tensor, spec: ModelSpec, *, n_pass: int = 1,
                     dropout: bool = False, seed: int = 0, window_offset: int = 0, pass_offset: int = 0,
                     logits: bool = False) -> torch.Tensor:
    """(members, n_pass, N) probabilities (or logits) of the pooled / single-channel CNN at fp32 on
    ``csrc/fused_tiled_x3.hip`` (BN on the moving statistics).  Launches hold < 2^31 samples; masks
    are keyed by the global (pass, window) ids, so splitting does not change the result."""
    o = _ext.ops()
    net = tiled_net(spec)
    if blobs.dim() == 1:
        blobs = blobs.unsqueeze(0)
    thr, _ = dropout_tables(spec)
    s63 = int(seed) & ((1 << 63) - 1)
    x = x.to(torch.float32).contiguous()
    n = x.shape[0]
    if not dropout:  # deterministic: every pass is identical
        y = o.fused_tiled_x3_forward(x, blobs, net, 1, int(window_offset), 0, s63, False, bool(logits), thr)
        return y.expand(blobs.shape[0], n_pass, n).contiguous()
    out = torch.empty(blobs.shape[0], n_pass, n, dtype=torch.float32, device=x.device)
    wc = min(n, _MAX_SAMPLES // 2)
    pc = max(1, (_MAX_SAMPLES // 2) // max(wc, 1))
    for w0 in range(0, n, wc):
        w1 = min(n, w0 + wc)
        for p0 in range(0, n_pass, pc):
            p1 = min(n_pass, p0 + pc)
            out[:, p0:p1, w0:w1] = o.fused_tiled_x3_forward(x[w0:w1], blobs, net, p1 - p0, int(window_offset) + w0,
                                                            int(pass_offset) + p0, s63, True, bool(logits), thr)
    return out


_MAX_SAMPLES = 1 << 31  # samples per fused launch (32-bit sample index); tests lower it


def dropout_tables(spec: ModelSpec):
    thr = [rng.dropout_threshold(b.dropout) for b in spec.blocks]
    dsc = [1.0 / (1.0 - b.dropout) if b.dropout < 1.0 else 0.0 for b in spec.blocks]
    return thr, dsc


def fused_forward(x_bf16: torch.Tensor, blobs: torch.Tensor, spec: ModelSpec = DEFAULT_SPEC, *, n_pass: int = 1,
                  dropout: bool = False, seed: int = 0, window_offset: int = 0, pass_offset: int = 0,
                  logits: bool = False) -> torch.Tensor:
    """Run the fused kernel: returns (members, n_pass, N) fp32 probabilities (or logits).

    One launch indexes samples (pass, window) with 32-bit ints, so a call with
    n_pass * N >= 2^31 samples is split into pass chunks (and window chunks if N alone is that
    large); masks are keyed by the global (pass, window) ids, so the result is that of one launch."""
    o = _ext.ops()
    if blobs.dim() == 1:
        blobs = blobs.unsqueeze(0)
    thr, dsc = dropout_tables(spec)
    seed = int(seed) & ((1 << 63) - 1)
    n_win = x_bf16.shape[0]
    if n_pass * n_win < _MAX_SAMPLES:
        return o.fused_forward(x_bf16, blobs, int(n_pass), int(window_offset), int(pass_offset), seed, bool(dropout),
                               bool(logits), thr, dsc, 0)
    out = torch.empty(blobs.shape[0], n_pass, n_win, dtype=torch.float32, device=x_bf16.device)
    wc = min(n_win, _MAX_SAMPLES - 1)
    pc = max(1, (_MAX_SAMPLES - 1) // wc)
    for w0 in range(0, n_win, wc):
        w1 = min(n_win, w0 + wc)
        for p0 in range(0, n_pass, pc):
            p1 = min(n_pass, p0 + pc)
            out[:, p0:p1, w0:w1] = o.fused_forward(x_bf16[w0:w1], blobs, p1 - p0, int(window_offset) + w0,
                                                   int(pass_offset) + p0, seed, bool(dropout), bool(logits), thr, dsc, 0)
    return out


# ------------------------------------------------------------------------------------------------
# CPU emulation of the kernel's arithmetic (bf16 operands, fp32 accumulate) straight from a blob.
# Used by the CPU test tier to validate the packing and by the GPU tier as a tighter oracle.
# ------------------------------------------------------------------------------------------------
def emulate_blob_forward(blob: torch.Tensor, x: torch.Tensor, spec: ModelSpec = DEFAULT_SPEC, *, dropout: bool = False,
                         seed: int = 0, pass_id: int = 0, sample_ids: Optional[torch.Tensor] = None,
                         logits: bool = False) -> torch.Tensor:
    from ..models.reference import conv1d_same

    lay = layout()
    blob = blob.cpu()
    ch, ks = FUSED_CHANNELS, FUSED_KSIZES
    n = x.shape[0]
    if sample_ids is None:
        sample_ids = torch.arange(n)
    h = x.float().to(torch.bfloat16).float()
    for l in range(6):
        nstep = (ch[l] * ks[l] + 31) // 32
        nbytes = nstep * (ch[l + 1] // 16) * 1024
        fr = blob[lay["woff"][l]: lay["woff"][l] + nbytes].view(torch.bfloat16).reshape(nstep, ch[l + 1] // 16, 64, 8)
        w = unpack_conv_fragments(fr, ks[l], ch[l], ch[l + 1])
        epi = blob[lay["eoff"][l]: lay["eoff"][l] + 4 * EPI_ROWS * ch[l + 1]].view(torch.float32).reshape(EPI_ROWS, ch[l + 1])
        y = conv1d_same(h, w, torch.zeros(ch[l + 1]))
        y = torch.minimum(torch.maximum(y * epi[0] + epi[1], epi[2]), epi[3])  # rows 4-7: same x 1/(1-rate)
        if dropout:
            y = rng.dropout_apply_torch(y, rng.stream_key(seed, l, pass_id), sample_ids, spec.blocks[l].dropout)
        h = y if l == 5 else y.to(torch.bfloat16).float()
    head = blob[lay["dense"]: lay["dense"] + 4 * (ch[6] + 1)].view(torch.float32)
    logit = h.mean(dim=1) @ head[: ch[6]] + head[ch[6]]
    return logit if logits else torch.sigmoid(logit)
