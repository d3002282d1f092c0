"""Diagnostic: gx3 conv (forward / dgrad) and wgrad on given shapes vs float64."""
import sys

import torch

sys.path.insert(0, ".")
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext  # noqa: E402
from tests.test_fp32_gpu import _conv64  # noqa: E402

o = _ext.ops()
dev = "cuda"
for (n, L, cin, cout, k) in [(64, 60, 224, 96, 7), (64, 60, 192, 224, 3), (64, 60, 96, 256, 9), (9, 60, 64, 48, 5),
                             (64, 7, 224, 96, 7)]:
    g = torch.Generator().manual_seed(1)
    p = (k - 1) // 2
    rs = L + 2 * p
    x = torch.randn(n, L, cin, generator=g)
    w = torch.randn(k, cin, cout, generator=g) * 0.05
    b = torch.randn(cout, generator=g) * 0.1
    xin = torch.zeros(2 * p + n * rs, cin, device=dev)
    xin[p: p + n * rs].view(n, rs, cin)[:, p: p + L].copy_(x)
    fwd = torch.empty(2 * ((k * cin + 31) // 32) * 512 * ((cout + 15) // 16), dtype=torch.float16, device=dev)
    dgr = torch.empty(2 * ((k * cout + 31) // 32) * 512 * ((cin + 15) // 16), dtype=torch.float16, device=dev)
    wsc = torch.ones(4, device=dev)
    part = torch.empty(16, device=dev)
    o.gx3_pack([w.to(dev).contiguous()], [fwd], [dgr], [wsc[:1]], [k], [cin], [cout], part)
    y = torch.empty(n * L, cout, device=dev)
    st = torch.zeros(16 * 2 * cout, device=dev)
    amax = torch.zeros(2, dtype=torch.int32, device=dev)
    o.gx3_conv(xin, fwd, wsc[:1], b.to(dev), y, st, amax[0:1], n, L, cin, cout, k, 1, rs, 2 * p, False)
    ref = _conv64(x, w, b, True).reshape(n * L, cout)
    ef = ((y.cpu().double() - ref).abs().max() / ref.abs().max()).item()
    dz = torch.randn(n, L, cout, generator=g)
    dzp = torch.zeros(n * rs, cout, device=dev)
    dzp.view(n, rs, cout)[:, p: p + L].copy_(dz)
    dh = torch.empty(n * L, cin, device=dev)
    o.gx3_conv(dzp, dgr, wsc[:1], None, dh, None, amax[1:2], n, L, cout, cin, k, 2, rs, p, False)
    ref = _conv64(dz, w.flip(0).permute(0, 2, 1).contiguous(), None, False).reshape(n * L, cin)
    err = (dh.cpu().double() - ref).abs()
    ed = (err.max() / ref.abs().max()).item()
    bad = (err > 1e-5 * ref.abs().max()).nonzero()
    gw = torch.empty(k, cin, cout, device=dev)
    wpart = torch.empty(64 * k * cin * cout, device=dev)
    o.gx3_wgrad(xin, dzp, amax[0:1], amax[1:2], n * rs, cin, cout, k, gw, wpart)
    xp, dzc = xin.cpu().double(), dzp.cpu().double()
    ref = torch.stack([xp[t: t + n * rs].t() @ dzc for t in range(k)])
    ew = ((gw.cpu().double() - ref).abs().max() / ref.abs().max()).item()
    print((n, L, cin, cout, k), f"fwd {ef:.2e} dgrad {ed:.2e} wgrad {ew:.2e} bad-dgrad {len(bad)}",
          bad[:5].tolist() if len(bad) else "")
