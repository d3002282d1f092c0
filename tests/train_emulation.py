"""Host emulation of the HIP training step's dataflow (same bf16 quantisation points, fp32 math).

Used by the GPU tests as a tight oracle for ``csrc/train_conv.hip``: the fp32 autograd reference
differs from any bf16 pipeline by quantisation noise that the BatchNorm backward amplifies
(gradients there are small residuals of large terms), so the kernels are checked against this
emulation with tight tolerances and against autograd only for direction (cosine similarity).
"""
import torch
import torch.nn.functional as F

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.reference import conv1d_same
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import rng


def bf(t):
    return t.to(torch.bfloat16).float()


def emulate_step(spec, p, x, y, seed, pass_id):
    """Returns (loss_sum, logits, grads dict, new moving stats dict)."""
    n = x.shape[0]
    L = x.shape[1]
    sid = torch.arange(n, device=x.device)
    cnt = n * L
    A = [bf(x)]
    R, S, masks = [], [], []
    for l, b in enumerate(spec.blocks):
        i = l + 1
        W = bf(p[f"conv1d_{i}/kernel"])
        Z = conv1d_same(A[-1], W, p[f"conv1d_{i}/bias"])
        Rl = bf(torch.relu(Z))
        mean = Rl.sum((0, 1)) / cnt
        var = (Rl * Rl).sum((0, 1)) / cnt - mean * mean
        rstd = torch.rsqrt(var.clamp_min(0) + spec.bn_epsilon)
        s = p[f"batchnorm_{i}/gamma"] * rstd
        t = p[f"batchnorm_{i}/beta"] - mean * s
        keep = rng.keep_mask_torch(rng.stream_key(seed, l, pass_id), sid, L, b.filters, b.dropout)
        dsc = 1.0 / (1.0 - b.dropout)
        Al = torch.where(keep, (Rl * s + t) * dsc, torch.zeros((), device=x.device))
        R.append(Rl)
        S.append((mean, var, rstd, s, t))
        masks.append((keep, dsc))
        A.append(bf(Al) if l < 5 else Al)  # block 6 output feeds the head in fp32
    G = A[-1].mean(1)
    w = p["output_layer/kernel"].reshape(-1)
    z = G @ w + p["output_layer/bias"]
    loss = (torch.clamp(z, min=0) - z * y + torch.log1p(torch.exp(-z.abs()))).sum()
    dl = (torch.sigmoid(z) - y) / n
    g = {"output_layer/kernel": (dl[:, None] * G).sum(0).reshape(-1, 1), "output_layer/bias": dl.sum().reshape(1)}
    keep6, dsc6 = masks[5]
    dY = torch.where(keep6, (dl[:, None, None] * w[None, None, :] / L) * dsc6, torch.zeros((), device=x.device))
    for l in range(5, -1, -1):
        i = l + 1
        mean, var, rstd, s, t = S[l]
        xh = (R[l] - mean) * rstd
        sdy = dY.sum((0, 1))
        sdyx = (dY * xh).sum((0, 1))
        g[f"batchnorm_{i}/beta"] = sdy
        g[f"batchnorm_{i}/gamma"] = sdyx
        gam = p[f"batchnorm_{i}/gamma"]
        dZ = bf(torch.where(R[l] > 0, gam * rstd * (dY - sdy / cnt - xh * sdyx / cnt), torch.zeros((), device=x.device)))
        g[f"conv1d_{i}/bias"] = dZ.sum((0, 1))
        k = spec.blocks[l].kernel_size
        pad = (k - 1) // 2
        Ap = F.pad(A[l].transpose(1, 2), (pad, k - 1 - pad)).transpose(1, 2)  # (n, L+k-1, Cin)
        gw = torch.stack([torch.einsum("ntc,ntd->cd", Ap[:, tap: tap + L], dZ) for tap in range(k)])
        g[f"conv1d_{i}/kernel"] = gw
        if l > 0:
            W = bf(p[f"conv1d_{i}/kernel"])
            # dA_{l-1}[t] = sum_tap dZ[t - tap + pad] W[tap]^T
            dZp = F.pad(dZ.transpose(1, 2), (k - 1 - pad, pad)).transpose(1, 2)
            dA = sum(torch.einsum("ntd,cd->ntc", dZp[:, k - 1 - tap: k - 1 - tap + L], W[tap]) for tap in range(k))
            keep, dsc = masks[l - 1]
            dY = bf(torch.where(keep, dA * dsc, torch.zeros((), device=x.device)))
    new_stats = {}
    for l in range(6):
        i = l + 1
        mean, var = S[l][0], S[l][1]
        m = spec.bn_momentum
        new_stats[f"batchnorm_{i}/moving_mean"] = p[f"batchnorm_{i}/moving_mean"] * m + mean * (1 - m)
        new_stats[f"batchnorm_{i}/moving_variance"] = p[f"batchnorm_{i}/moving_variance"] * m + var.clamp_min(0) * (1 - m)
    return loss.item(), z, g, new_stats
