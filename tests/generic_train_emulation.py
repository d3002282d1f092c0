"""Host emulation of the generic HIP training step's dataflow (``ops/generic_train.py``) for any
ModelSpec, pooled blocks included: the same bf16 quantisation points as the kernels, fp32 math.

Quantisation points: input, conv weights, the stored pre-BN activation z, every block output
(the next block's input / the head input), dz, and the dgrad output are bf16; BN moments come from
the fp32 relu output, the bias gradient from the unrounded dz, wgrad accumulates bf16 operands in
fp32.  The fp32 autograd reference differs from this by quantisation noise that the BatchNorm
backward amplifies, so the GPU test checks the kernels tightly against this emulation and only
for direction against autograd (as ``train_emulation.py`` does for the reference architecture).
"""
import torch
import torch.nn.functional as F

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.reference import conv1d_same
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import rng


def bf(t):
    return t.to(torch.bfloat16).float()


def _pool_pairs(y):
    n, L, c = y.shape
    lo = L // 2
    ya, yb = y[:, 0: 2 * lo: 2], y[:, 1: 2 * lo: 2]
    return torch.maximum(ya, yb), ya >= yb


def emulate_generic_step(spec, p, x, y, seed, pass_id):
    """Returns (loss_sum, logits, grads dict, new moving stats dict)."""
    n = x.shape[0]
    dev = x.device
    sid = torch.arange(n, device=dev)
    A = [bf(x)]
    S = []
    lengths = spec.lengths()
    for l, b in enumerate(spec.blocks):
        i = l + 1
        L = lengths[l]
        W = bf(p[f"conv1d_{i}/kernel"])
        R32 = torch.relu(conv1d_same(A[-1], W, p[f"conv1d_{i}/bias"]))
        cnt = n * L
        mean = R32.sum((0, 1)) / cnt
        var = ((R32 * R32).sum((0, 1)) / cnt - mean * mean).clamp_min(0)
        rstd = torch.rsqrt(var + spec.bn_epsilon)
        s = p[f"batchnorm_{i}/gamma"] * rstd
        t = p[f"batchnorm_{i}/beta"] - mean * s
        Z = bf(R32)
        Y = Z * s + t
        win = None
        if b.pool:
            Y, win = _pool_pairs(Y)
        lo = Y.shape[1]
        keep = rng.keep_mask_torch(rng.stream_key(seed, l, pass_id), sid, lo, b.filters, b.dropout)
        dsc = 1.0 / (1.0 - b.dropout)
        if b.dropout > 0:
            Y = torch.where(keep, Y * dsc, torch.zeros((), device=dev))
        S.append((Z, mean, var, rstd, win, keep, dsc))
        A.append(bf(Y))
    G = A[-1].mean(1)
    w = p["output_layer/kernel"].reshape(-1)
    z = G @ w + p["output_layer/bias"]
    loss = (torch.clamp(z, min=0) - z * y + torch.log1p(torch.exp(-z.abs()))).sum()
    dl = (torch.sigmoid(z) - y) / n
    g = {"output_layer/kernel": (dl[:, None] * G).sum(0).reshape(-1, 1), "output_layer/bias": dl.sum().reshape(1)}
    dH = dl[:, None, None] * w[None, None, :] / A[-1].shape[1] * torch.ones_like(A[-1])
    for l in range(len(spec.blocks) - 1, -1, -1):
        i = l + 1
        b = spec.blocks[l]
        L = lengths[l]
        cnt = n * L
        Z, mean, var, rstd, win, keep, dsc = S[l]
        dY = torch.where(keep, dH * dsc, torch.zeros((), device=dev)) if b.dropout > 0 else dH
        if b.pool:
            full = torch.zeros(n, L, dY.shape[2], device=dev)
            lo = dY.shape[1]
            full[:, 0: 2 * lo: 2] = torch.where(win, dY, torch.zeros((), device=dev))
            full[:, 1: 2 * lo: 2] = torch.where(win, torch.zeros((), device=dev), dY)
            dY = full
        xh = (Z - mean) * rstd
        sdy = dY.sum((0, 1))
        sdyx = (dY * xh).sum((0, 1))
        g[f"batchnorm_{i}/beta"] = sdy
        g[f"batchnorm_{i}/gamma"] = sdyx
        gam = p[f"batchnorm_{i}/gamma"]
        dZ32 = torch.where(Z > 0, gam * rstd * (dY - sdy / cnt - xh * sdyx / cnt), torch.zeros((), device=dev))
        g[f"conv1d_{i}/bias"] = dZ32.sum((0, 1))
        dZ = bf(dZ32)
        k = b.kernel_size
        pad = (k - 1) // 2
        Ap = F.pad(A[l].transpose(1, 2), (pad, k - 1 - pad)).transpose(1, 2)
        g[f"conv1d_{i}/kernel"] = torch.stack([torch.einsum("ntc,ntd->cd", Ap[:, tap: tap + L], dZ) for tap in range(k)])
        if l > 0:
            W = bf(p[f"conv1d_{i}/kernel"])
            dZp = F.pad(dZ.transpose(1, 2), (k - 1 - pad, pad)).transpose(1, 2)
            dH = bf(sum(torch.einsum("ntd,cd->ntc", dZp[:, k - 1 - tap: k - 1 - tap + L], W[tap]) for tap in range(k)))
    new_stats = {}
    m = spec.bn_momentum
    for l in range(len(spec.blocks)):
        i = l + 1
        mean, var = S[l][1], S[l][2]
        new_stats[f"batchnorm_{i}/moving_mean"] = p[f"batchnorm_{i}/moving_mean"] * m + mean * (1 - m)
        new_stats[f"batchnorm_{i}/moving_variance"] = p[f"batchnorm_{i}/moving_variance"] * m + var * (1 - m)
    return loss.item(), z, g, new_stats
