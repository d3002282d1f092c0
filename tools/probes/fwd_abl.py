"""Time one batch-statistics MC-Dropout chunk (16 passes x 16384 windows) through the layer-wise
forward kernels; used with probe builds of the extension (-DAPNEAUQ_FWD_ABL=bits)."""
import json
import sys

import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops

tag = sys.argv[1] if len(sys.argv) > 1 else "0"
dev = torch.device("cuda", 0)
m = AlarconCNN1D(seed=1, device=dev, params={k: v.to(dev) for k, v in R.synthetic_params(DEFAULT_SPEC, 1).items()})
x = torch.randn(16384, 60, 4, generator=torch.Generator().manual_seed(0)).to(dev)
run = lambda i: train_ops.forward_batch_stats(m, x, 16, pass_base=16 * i, seed=3, update_moving=False,
                                              max_samples=1 << 18)
run(0)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(5):
    run(i + 1)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"abl": tag, "ms_per_chunk": round(e0.elapsed_time(e1) / 5, 3)}), flush=True)
