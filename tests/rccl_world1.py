"""RCCL ("nccl" backend) collectives on device tensors at world size 1 — run as a subprocess by
tests/test_rccl_gpu.py (a one-GPU box cannot host two RCCL ranks, but world 1 exercises the same
init / device binding / collective code paths the multi-GPU runs use).

Prints one JSON line with the checks' results."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["APNEAUQ_FORCE_PG"] = "1"
for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
    os.environ.pop(k, None)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as S  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import dist as pdist  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import inference as pinf  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import distributed as uqd  # noqa: E402

info = pdist.init()
out = {"backend": info.backend, "pg_backend": dist.get_backend(), "device": str(info.device),
       "world": dist.get_world_size()}
dev = info.device
t = torch.arange(8, dtype=torch.float32, device=dev)
dist.all_reduce(t)
out["all_reduce"] = bool(torch.equal(t, torch.arange(8, dtype=torch.float32, device=dev)))
bufs = [torch.empty(4, device=dev)]
dist.all_gather(bufs, torch.full((4,), 3.0, device=dev))
out["all_gather"] = bool((bufs[0] == 3).all())
p = torch.rand(2, 10, device=dev)
out["all_to_all_members"] = bool(torch.equal(pinf.all_to_all_members(p, 1), p))
send = torch.arange(6, dtype=torch.float32, device=dev)
recv = torch.empty_like(send)
dist.all_to_all_single(recv, send)
out["all_to_all_single"] = bool(torch.equal(recv, send))
# SyncBN batch-statistics MC Dropout with the RCCL all-reduce as the sync: equals the unsynced run
params = {k: v.to(dev) for k, v in R.synthetic_params(S, 5).items()}
x = torch.randn(64, 60, 4, device=dev).to(torch.bfloat16)
m1 = AlarconCNN1D(seed=5, device=dev, params={k: v.clone() for k, v in params.items()})
m2 = AlarconCNN1D(seed=5, device=dev, params={k: v.clone() for k, v in params.items()})
a = train_ops.forward_batch_stats(m1, x, 3, pass_base=0, seed=9, update_moving=False)
b = train_ops.forward_batch_stats(m2, x, 3, pass_base=0, seed=9, update_moving=False,
                                  sync=lambda z: dist.all_reduce(z), global_n=64)
out["syncbn_max_abs_diff"] = float((a - b).abs().max())
ga = uqd._gather_windows(torch.rand(3, 64, device=dev), 64, 1)
out["gather_windows_shape"] = list(ga.shape)
out["devices"] = pdist.gather_device_ids()
torch.cuda.synchronize()
pdist.shutdown()
print(json.dumps(out), flush=True)
