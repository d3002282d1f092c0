"""Batch-BN MC Dropout: one launch sequence over all CUs vs the passes split in two halves on two HIP
streams with half-size persistent grids (the two sequences' layers desynchronise, so HBM-heavy and
MFMA-heavy layers could share the chip)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import x3  # noqa: E402

dev = torch.device("cuda")
x = torch.randn(16384, 60, 4, generator=torch.Generator().manual_seed(1)).to(dev)
p = {k: v.to(dev) for k, v in R.synthetic_params(SPEC, 1).items()}
m1 = x3.X3Model(SPEC, [{k: v.clone() for k, v in p.items()}])
m2 = x3.X3Model(SPEC, [{k: v.clone() for k, v in p.items()}])
ncu = torch.cuda.get_device_properties(0).multi_processor_count
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def one():
    return x3.mcd_batch(m1, x, 50, seed=1, update_moving=False)


def two(split):
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        a = x3.mcd_batch(m1, x, 25, seed=1, pass_base=0, update_moving=False, grid=split)
    with torch.cuda.stream(s2):
        b = x3.mcd_batch(m2, x, 25, seed=1, pass_base=25, update_moving=False, grid=ncu - split)
    torch.cuda.current_stream().wait_stream(s1)
    torch.cuda.current_stream().wait_stream(s2)
    return torch.cat([a, b])


def timeit(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return round(min(ts), 2)


ref = one()
alt = two(ncu // 2)
print(json.dumps({"max_abs_diff": float((ref - alt).abs().max())}), flush=True)
for r in range(2):
    print(json.dumps({"one_stream_ms": timeit(one), "two_streams_half_grid_ms": timeit(lambda: two(ncu // 2))}),
          flush=True)
