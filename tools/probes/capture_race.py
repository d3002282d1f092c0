"""First replay of a freshly captured training graph vs the eager step (fresh model each time), for
the reference-spec HIP path and the generic (pooled) path.  Run with APNEAUQ_CAPTURE_SYNC=0 to check
that no replay depends on the post-capture device synchronize."""
import collections
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_generic_gpu import SPECS  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
bad = 0
for name, spec in (("reference", DEFAULT_SPEC), ("pooled", SPECS["pooled"])):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(256, spec.input_length, spec.input_channels, generator=g).cuda()
    y = (torch.rand(256, generator=g) < 0.4).float().cuda()
    for mode in ("0", "1"):
        os.environ["APNEAUQ_TRAIN_GRAPH"] = mode
        seen = collections.Counter()
        for rep in range(reps if mode == "1" else 3):  # noqa: B007
            m = AlarconCNN1D(spec=spec, seed=4, device="cuda")
            l1 = round(float(m.train_step(x[:64], y[:64])), 3)
            l2 = round(float(m.train_step(x[64:128], y[64:128])), 3)
            seen[(l1, l2)] += 1
            del m
            gc.collect()
        print(name, "graph" if mode == "1" else "eager", dict(seen), flush=True)
        if len(seen) > 1:
            bad += 1
sys.exit(1 if bad else 0)
