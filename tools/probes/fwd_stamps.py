"""Phase timeline of the batch-BN forward kernel (probe build -DAPNEAUQ_FWD_STAMPS=<layer>).

Runs one 16-pass x 16384-window batch-statistics MC-Dropout chunk, reads the s_memtime stamps of the
first 1024 workgroups x 16 tiles of the instrumented layer and reports per-phase medians and how the
phases of two workgroups sharing a CU overlap (is the co-resident workgroup's conv running while this
one stages / copies out?)."""
import json
import sys

import numpy as np
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, train_ops

WG, T, N = 1024, 16, 6
dev = torch.device("cuda", 0)
m = AlarconCNN1D(seed=1, device=dev, params={k: v.to(dev) for k, v in R.synthetic_params(DEFAULT_SPEC, 1).items()})
x = torch.randn(16384, 60, 4, generator=torch.Generator().manual_seed(0)).to(dev)
for i in range(3):
    train_ops.forward_batch_stats(m, x, 16, pass_base=16 * i, seed=3, update_moving=False, max_samples=1 << 18)
torch.cuda.synchronize()
buf = torch.zeros(WG * 2 * 4 + WG * T * N * 8, dtype=torch.uint8)
rc = _ext.ops().train_stamps(buf)
assert rc == 0, f"not a stamps build (rc {rc})"
raw = buf.numpy().tobytes()
ids = np.frombuffer(raw[: WG * 8], dtype=np.uint32).reshape(WG, 2)
st = np.frombuffer(raw[WG * 8:], dtype=np.uint64).reshape(WG, T, N).astype(np.int64)
ok = (st > 0).all(axis=(1, 2))
names = ["stage", "conv", "bar1", "epi", "mom+copy"]
d = np.diff(st, axis=2)  # (WG, T, 5)
res = {"workgroups": int(ok.sum())}
res["median_cycles"] = {n: float(np.median(d[ok, 1:, i])) for i, n in enumerate(names)}
res["median_tile"] = float(np.median(st[ok, 2:, 0] - st[ok, 1:-1, 0]))
# co-resident pairs: same (xcc, cu) with overlapping lifetimes
key = [(int(a), int(b)) for a, b in ids]
by = {}
for w in range(WG):
    if ok[w]:
        by.setdefault(key[w], []).append(w)
fr_conv_conv, fr_stage_conv, fr_copy_conv, pairs = [], [], [], 0
def overlap(a0, a1, b0, b1):
    return max(0, min(a1, b1) - max(a0, b0))
for ws in by.values():
    for i in range(len(ws)):
        for j in range(len(ws)):
            if i == j:
                continue
            a, b = ws[i], ws[j]
            if st[b, 0, 0] > st[a, -1, 5] or st[a, 0, 0] > st[b, -1, 5]:
                continue
            pairs += 1
            bconv = [(st[b, k, 1], st[b, k, 2]) for k in range(T)]
            for k in range(1, T - 1):
                for (p0, p1, lst) in ((st[a, k, 1], st[a, k, 2], fr_conv_conv), (st[a, k, 0], st[a, k, 1], fr_stage_conv),
                                      (st[a, k, 4], st[a, k, 5], fr_copy_conv)):
                    tot = p1 - p0
                    if tot > 0:
                        lst.append(sum(overlap(p0, p1, c0, c1) for c0, c1 in bconv) / tot)
res["coresident_pairs"] = pairs // 2
res["frac_of_conv_overlapping_partner_conv"] = float(np.mean(fr_conv_conv)) if fr_conv_conv else None
res["frac_of_stage_overlapping_partner_conv"] = float(np.mean(fr_stage_conv)) if fr_stage_conv else None
res["frac_of_copy_overlapping_partner_conv"] = float(np.mean(fr_copy_conv)) if fr_copy_conv else None
print(json.dumps(res, indent=1), flush=True)
