"""Counter-based dropout masks shared bit-for-bit by the HIP kernels and the host reference.

The reference draws dropout masks from TensorFlow's stateful RNG inside every
``model(x, training=True)`` call (``uncertainty_quantification/uq_techniques.py:22``), so its
masks depend on call order and device.  Here a mask bit is a pure function of *global*
coordinates ``(seed, layer, pass, sample, t, channel)``: MC-Dropout results are therefore
identical whether the T x N samples run on one GPU or are sharded over eight, and the CPU
reference can regenerate exactly the mask a kernel used (SURVEY §7.3 "RNG determinism").

Definition (all arithmetic on uint32)::

    mix(x)        = lowbias32 integer hash (x^=x>>16; x*=0x7feb352d; x^=x>>15; x*=0x846ca68b; x^=x>>16)
    stream_key    = mix(mix(mix(mix(seed_lo ^ 0x68bc21eb) ^ seed_hi) ^ (layer*0x9e3779b9)) ^ pass)
    sample_key    = mix(stream_key ^ mix(sample + 0x2545f491))
    h             = mix(sample_key ^ ((t << 9) | (c >> 1)))
    u16           = (h >> 16) if c odd else (h & 0xffff)
    keep          = u16 >= thr16,     thr16 = round(rate * 65536)
    y             = keep ? x / (1 - rate) : 0          (inverted dropout, as Keras)

One 32-bit hash feeds two channels, which matches the MFMA accumulator layout of the fused
kernel where a lane owns one time step and four consecutive channels.
"""
from __future__ import annotations

import numpy as np
import torch

_M32 = 0xFFFFFFFF
GOLDEN = 0x9E3779B9


def mix32_int(x: int) -> int:
    x &= _M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & _M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & _M32
    x ^= x >> 16
    return x


def stream_key(seed: int, layer: int, pass_id: int) -> int:
    """32-bit key of one (seed, layer, pass) dropout stream (a host scalar, passed to kernels)."""
    k = mix32_int((seed & _M32) ^ 0x68BC21EB)
    k = mix32_int(k ^ ((seed >> 32) & _M32))
    k = mix32_int(k ^ ((layer * GOLDEN) & _M32))
    k = mix32_int(k ^ (pass_id & _M32))
    return k


def dropout_threshold(rate: float) -> int:
    return int(min(65536, max(0, round(rate * 65536.0))))


# ----------------------------------------------------------------------------- numpy
def _mix32_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32, copy=True)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def keep_mask_np(key: int, samples: np.ndarray, length: int, channels: int, rate: float) -> np.ndarray:
    """Boolean keep-mask of shape (len(samples), length, channels)."""
    samples = np.asarray(samples, dtype=np.uint64).astype(np.uint32)
    with np.errstate(over="ignore"):
        sk = _mix32_np(np.uint32(key) ^ _mix32_np(samples + np.uint32(0x2545F491)))
        t = np.arange(length, dtype=np.uint32)[:, None]
        c = np.arange(channels, dtype=np.uint32)[None, :]
        ctr = (t << np.uint32(9)) | (c >> np.uint32(1))
        h = _mix32_np(sk[:, None, None] ^ ctr[None])
    u16 = np.where((c & 1)[None].astype(bool), h >> np.uint32(16), h & np.uint32(0xFFFF))
    return u16 >= np.uint32(dropout_threshold(rate))


# ----------------------------------------------------------------------------- torch
def _mix32_t(x: torch.Tensor) -> torch.Tensor:
    # int64 arithmetic with explicit 32-bit wrap (torch has no uint32 multiply on every backend)
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def keep_mask_torch(key: int, samples: torch.Tensor, length: int, channels: int, rate: float) -> torch.Tensor:
    """Boolean keep-mask (len(samples), length, channels) on ``samples.device``."""
    dev = samples.device
    s = samples.to(torch.int64) & _M32
    sk = _mix32_t(torch.full_like(s, key) ^ _mix32_t(s + 0x2545F491))
    t = torch.arange(length, device=dev, dtype=torch.int64)[:, None]
    c = torch.arange(channels, device=dev, dtype=torch.int64)[None, :]
    ctr = (t << 9) | (c >> 1)
    h = _mix32_t(sk[:, None, None] ^ ctr[None])
    u16 = torch.where((c & 1).bool()[None], h >> 16, h & 0xFFFF)
    return u16 >= dropout_threshold(rate)


def dropout_apply_torch(x: torch.Tensor, key: int, samples: torch.Tensor, rate: float) -> torch.Tensor:
    """Inverted dropout on a channels-last (N, L, C) tensor with the counter-based mask."""
    if rate <= 0.0:
        return x
    keep = keep_mask_torch(key, samples, x.shape[1], x.shape[2], rate)
    return torch.where(keep, x * (1.0 / (1.0 - rate)), torch.zeros((), dtype=x.dtype, device=x.device))
