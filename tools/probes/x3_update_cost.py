"""Batch-BN MCD with / without the moving-average side effect and with a world-size-1 SyncBN hook, same box."""
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
m = x3.X3Model(SPEC, [p])


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


noop = lambda t: None  # noqa: E731
ms = x3._max_samples(dev, x3.BYTES_PER_SAMPLE)
for r in range(2):
    print(json.dumps({
        "update_false": timeit(lambda: x3.mcd_batch(m, x, 50, seed=1, update_moving=False)),
        "update_true": timeit(lambda: x3.mcd_batch(m, x, 50, seed=1, update_moving=True)),
        "update_true_sync_hook": timeit(lambda: x3.mcd_batch(m, x, 50, seed=1, update_moving=True, sync=noop, max_samples=ms,
                                                             global_n=16384)),
    }), flush=True)
