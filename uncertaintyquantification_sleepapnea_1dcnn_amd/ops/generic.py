"""Host side of the layer-wise HIP inference path for any :class:`ModelSpec` (``csrc/generic_conv.hip``).

The fused kernel (``ops/fused.py``) covers the reference architecture only.  Everything else the
spec can express -- the opt-in ``MaxPool1D(2)`` blocks (the thesis' pooled
``ensemble_cnn`` models), other window shapes such as the north-star "30 s single-channel"
``ModelSpec(30, 1)``, other filter counts and odd kernel sizes -- runs here: one MFMA launch per
block (bias + ReLU + BN(running) + pool + counter-based dropout fused into its epilogue) and one
GAP + Dense head launch, with bf16 activations between blocks.  Two variants of the reference CNN
instead run a fused whole-network kernel (``csrc/fused_tiled.hip``, multi-sample tiles, activations
in LDS, one launch; :func:`fused.tiled_net`): MaxPool1D after blocks 1-5, and the north star's 30 s
single-channel window.  ``APNEAUQ_TILED_FUSED=0`` forces the layer-wise kernels (A/B runs).

Dropout masks are the same pure function of (seed, layer, pass, window, t, channel) as everywhere
else (``ops/rng.py``), so results match the fp32 reference's masks exactly and do not depend on
chunking or sharding.  BatchNorm with batch statistics (``bn_mode="batch"``, training) runs on the
generic training kernels (``ops/generic_train.py``).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

from ..models.spec import ModelSpec
from . import _ext, fused, rng

# activations of one chunk are bounded to ~2^28 bf16 elements (512 MiB) per layer
_CHUNK_ELEMS = 1 << 28


def supports(spec: ModelSpec) -> bool:
    """Shapes the generic kernels handle: Cout % 4 == 0, odd kernels, C <= 1024 (dropout hash)."""
    ch = spec.channels()
    return (all(b.filters % 4 == 0 and b.kernel_size % 2 == 1 for b in spec.blocks)
            and max(ch) <= 1024 and spec.input_length < (1 << 22) and min(spec.lengths()) >= 1)


def pack(spec: ModelSpec, p) -> Dict[str, object]:
    """Per-block (A fragments, epilogue constants) + dense head, on the params' device."""
    dev = p["conv1d_1/kernel"].device
    blocks: List[Tuple[torch.Tensor, torch.Tensor]] = []
    for i, b in enumerate(spec.blocks, 1):
        w = p[f"conv1d_{i}/kernel"].float().to(dev)
        cout = w.shape[2]
        cpad = (cout + 15) // 16 * 16
        wp = torch.nn.functional.pad(w, (0, cpad - cout))
        fr = fused.pack_conv_fragments(wp)
        scale, shift = fused.bn_affine(spec, p, i)
        pad = lambda v: torch.nn.functional.pad(v.float().to(dev), (0, cpad - cout))  # noqa: E731
        epi = fused.epilogue_constants(pad(p[f"conv1d_{i}/bias"]), pad(scale), pad(shift))
        epi = torch.cat([epi, epi * (1.0 / (1.0 - b.dropout) if b.dropout < 1.0 else 0.0)]).contiguous()
        blocks.append((fr, epi))
    dense_w = p["output_layer/kernel"].float().reshape(-1).to(dev).contiguous()
    dense_b = float(p["output_layer/bias"].float().reshape(-1)[0])
    out = {"blocks": blocks, "dense_w": dense_w, "dense_b": dense_b}
    if _tiled_enabled(spec):
        out["tiled_blob"] = fused.pack_blob(spec, p).unsqueeze(0)
    return out


def _tiled_enabled(spec: ModelSpec) -> bool:
    return fused.tiled_net(spec) is not None and os.environ.get("APNEAUQ_TILED_FUSED", "1") != "0"


_MAX_SAMPLES = 1 << 31  # samples per fused-tiled launch (32-bit sample / tile ids)


def _tiled_forward(packed, spec: ModelSpec, x: torch.Tensor, n_pass: int, dropout: bool, seed: int,
                   window_offset: int, pass_offset: int, logits: bool) -> torch.Tensor:
    """(n_pass, N) through ``csrc/fused_tiled.hip``; launches split so that one holds < 2^31 samples
    (masks are keyed by global pass / window ids, so the split does not change the result)."""
    o = _ext.ops()
    launch = o.fused_pooled_forward if fused.tiled_net(spec) == 0 else o.fused_single_forward
    thr, dsc = fused.dropout_tables(spec)
    s63 = int(seed) & ((1 << 63) - 1)
    blob = packed["tiled_blob"]
    n = x.shape[0]
    if not dropout:  # deterministic: every pass is identical
        y = launch(x, blob, 1, int(window_offset), 0, s63, False, bool(logits), thr, dsc)[0, 0]
        return y.unsqueeze(0).expand(n_pass, n).contiguous()
    out = torch.empty(n_pass, n, dtype=torch.float32, device=x.device)
    wc = min(n, _MAX_SAMPLES // 2)
    pc = max(1, (_MAX_SAMPLES // 2) // wc)
    for w0 in range(0, n, wc):
        w1 = min(n, w0 + wc)
        for p0 in range(0, n_pass, pc):
            p1 = min(n_pass, p0 + pc)
            out[p0:p1, w0:w1] = launch(x[w0:w1], blob, p1 - p0, int(window_offset) + w0, int(pass_offset) + p0, s63,
                                       True, bool(logits), thr, dsc)[0]
    return out


def _forward_chunk(packed, spec: ModelSpec, x_bf16: torch.Tensor, n_win: int, dropout: bool, seed: int,
                   pass_offset: int, window_offset: int, logits: bool) -> torch.Tensor:
    o = _ext.ops()
    h = x_bf16
    thr, _ = fused.dropout_tables(spec)
    s63 = int(seed) & ((1 << 63) - 1)
    for l, (b, (fr, epi)) in enumerate(zip(spec.blocks, packed["blocks"])):
        drop = bool(dropout and b.dropout > 0)
        h = o.generic_conv(h, fr, epi, b.filters, b.kernel_size, bool(b.pool), drop, int(thr[l]), l, int(n_win),
                           int(pass_offset), int(window_offset), s63)
    return o.generic_head(h, packed["dense_w"], packed["dense_b"], bool(logits))


def forward(packed, spec: ModelSpec, x_bf16: torch.Tensor, *, n_pass: int = 1, dropout: bool = False, seed: int = 0,
            window_offset: int = 0, pass_offset: int = 0, logits: bool = False) -> torch.Tensor:
    """(n_pass, N) fp32 probabilities (or logits) of one model; passes are chunked to bound memory."""
    if not supports(spec):
        raise ValueError("generic HIP path: unsupported architecture (needs filters % 4 == 0, odd kernels)")
    n = x_bf16.shape[0]
    out = torch.empty(n_pass, n, dtype=torch.float32, device=x_bf16.device)
    if n == 0:
        return out
    x = x_bf16.contiguous()
    if "tiled_blob" in packed:
        return _tiled_forward(packed, spec, x, n_pass, dropout, seed, window_offset, pass_offset, logits)
    widest = max(ln * c for ln, c in zip(spec.lengths(), spec.channels()))
    per_pass = max(1, n * widest)
    pc = max(1, min(n_pass, _CHUNK_ELEMS // per_pass))
    if not dropout:  # deterministic: every pass is identical
        out[:] = _forward_chunk(packed, spec, x, n, False, seed, pass_offset, window_offset, logits)
        return out
    if pc == 1 and n * widest > _CHUNK_ELEMS:  # one pass is itself too big: split the windows
        step = max(1, _CHUNK_ELEMS // widest)
        for t in range(n_pass):
            for s in range(0, n, step):
                xe = x[s:s + step]
                out[t, s:s + step] = _forward_chunk(packed, spec, xe, xe.shape[0], True, seed, pass_offset + t,
                                                    window_offset + s, logits)
        return out
    for p0 in range(0, n_pass, pc):
        k = min(pc, n_pass - p0)
        xr = x.repeat(k, 1, 1) if k > 1 else x
        out[p0:p0 + k] = _forward_chunk(packed, spec, xr, n, True, seed, pass_offset + p0, window_offset,
                                        logits).reshape(k, n)
    return out


def emulate(spec: ModelSpec, p, x: torch.Tensor, *, dropout: bool = False, seed: int = 0, pass_id: int = 0,
            sample_ids: Optional[torch.Tensor] = None, logits: bool = False,
            last_fp32: Optional[bool] = None) -> torch.Tensor:
    """CPU emulation of the generic kernels' arithmetic (bf16 operands and activations, fp32
    accumulation, folded epilogue) -- the tight oracle for the GPU tests.  ``last_fp32``: the last
    block's output feeds the head in fp32 (the fused kernels; default: whenever :func:`forward`
    takes a fused kernel for ``spec``)."""
    if last_fp32 is None:
        last_fp32 = _tiled_enabled(spec)
    from ..models.reference import conv1d_same

    n = x.shape[0]
    if sample_ids is None:
        sample_ids = torch.arange(n)
    h = x.float().to(torch.bfloat16).float()
    for i, b in enumerate(spec.blocks, 1):
        w = p[f"conv1d_{i}/kernel"].float().to(torch.bfloat16).float()
        scale, shift = fused.bn_affine(spec, p, i)
        epi = fused.epilogue_constants(p[f"conv1d_{i}/bias"].float(), scale, shift)
        if dropout and b.dropout > 0:
            epi = epi * (1.0 / (1.0 - b.dropout))
        y = conv1d_same(h, w, torch.zeros(b.filters))
        y = torch.minimum(torch.maximum(y * epi[0] + epi[1], epi[2]), epi[3])
        if b.pool:
            y = torch.nn.functional.max_pool1d(y.transpose(1, 2), 2).transpose(1, 2)
        if dropout and b.dropout > 0:
            keep = rng.keep_mask_torch(rng.stream_key(seed, i - 1, pass_id), sample_ids, y.shape[1], y.shape[2],
                                       b.dropout)
            y = torch.where(keep, y, torch.zeros_like(y))
        h = y if (last_fp32 and i == len(spec.blocks)) else y.to(torch.bfloat16).float()
    logit = h.mean(dim=1) @ p["output_layer/kernel"].float().reshape(-1) + p["output_layer/bias"].float().reshape(-1)
    return logit if logits else torch.sigmoid(logit)
