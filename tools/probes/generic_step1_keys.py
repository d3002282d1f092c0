"""Generic graph step 1: losses with forced device keys (stale-key hypothesis) and with a device
sync before the first replay."""
import collections
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_generic_gpu import SPECS  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import generic_train as GT  # noqa: E402

gc.disable()  # an old graph destroyed by a collection during another capture aborts (probe only)
spec = SPECS["pooled"]
g = torch.Generator().manual_seed(3)
x = torch.randn(256, spec.input_length, spec.input_channels, generator=g).cuda()
y = (torch.rand(256, generator=g) < 0.4).float().cuda()
os.environ["APNEAUQ_TRAIN_GRAPH"] = "1"
orig_replay = torch.cuda.CUDAGraph.replay


def run(tag, n):
    seen = collections.Counter()
    for rep in range(n):
        m = AlarconCNN1D(spec=spec, seed=4, device="cuda")
        seen[round(float(m.train_step(x[:64], y[:64])), 4)] += 1
        del m
        gc.collect()
    print(tag, dict(seen), flush=True)


# zero keys for every layer / for layer 0 only
for which in ("all", "l0"):
    def replay(self, which=which):
        step = [s for s in GT.__dict__.values() if False]
        return orig_replay(self)
    gcall = GT.GraphedGenericStep.__call__

    def patched(self, xx, yy, which=which, gcall=gcall):
        orig_copy = self.keys.copy_

        def zcopy(src):
            src = src.clone()
            if which == "all":
                src.zero_()
            else:
                src[0] = 0
            return orig_copy(src)
        self.keys.copy_ = zcopy
        try:
            return gcall(self, xx, yy)
        finally:
            del self.keys.copy_
    GT.GraphedGenericStep.__call__ = patched
    run("zero-keys-" + which, 1)
    GT.GraphedGenericStep.__call__ = gcall


def sync_replay(self):
    torch.cuda.synchronize()
    return orig_replay(self)


run("as-is", 40)
torch.cuda.CUDAGraph.replay = sync_replay
run("sync-before-replay", 40)
