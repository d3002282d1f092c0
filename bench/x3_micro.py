"""Timing of the fp32-faithful (fp16x3) engine phases on one GPU (builder probe, not the headline).

``python -m bench.x3_micro [--windows N] [--passes T] [--members M] [--reps R]``: batch-BN MC Dropout
(T passes over N windows), Deep-Ensemble predict (M members) and standard MC Dropout, each timed with
events after a warmup; prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=16384)
    ap.add_argument("--passes", type=int, default=50)
    ap.add_argument("--members", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="comma list of mcd,de,run")
    a = ap.parse_args(argv)
    import torch

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import x3

    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(a.windows, 60, 4, generator=g).to(dev)
    only = set(a.only.split(",")) if a.only else {"mcd", "de", "run"}
    out = {"windows": a.windows, "passes": a.passes, "members": a.members}

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return min(ts), sorted(ts)[len(ts) // 2]

    flop = 2 * SPEC.forward_macs()
    if "mcd" in only:
        m = x3.X3Model(SPEC, [{k: v.to(dev) for k, v in R.synthetic_params(SPEC, 1).items()}])
        best, med = timeit(lambda: x3.mcd_batch(m, x, a.passes, seed=1, update_moving=True))
        out["mcd_batch_ms"] = [round(best, 3), round(med, 3)]
        out["mcd_batch_tflops"] = round(a.windows * a.passes * flop / (best / 1e3) / 1e12, 1)
    if "de" in only:
        m = x3.X3Model(SPEC, [{k: v.to(dev) for k, v in R.synthetic_params(SPEC, 100 + i).items()}
                              for i in range(a.members)])
        best, med = timeit(lambda: x3.forward_running(m, x))
        out["de_ms"] = [round(best, 3), round(med, 3)]
        out["de_tflops"] = round(a.windows * a.members * flop / (best / 1e3) / 1e12, 1)
    if "run" in only:
        m = x3.X3Model(SPEC, [{k: v.to(dev) for k, v in R.synthetic_params(SPEC, 1).items()}])
        best, med = timeit(lambda: x3.forward_running(m, x, n_pass=a.passes, dropout=True, seed=3))
        out["mcd_running_ms"] = [round(best, 3), round(med, 3)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
