"""Probe driver: per-wave phase cycle split of the x3 layer kernels from an X3_PROF build
(APNEAUQ_SO_PATH=gpuprobe/prof.so python tools/x3_prof_run.py)."""
import ctypes
import os
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC  # noqa: E402
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, x3  # noqa: E402

_ext.require()
lib = ctypes.CDLL(os.environ["APNEAUQ_SO_PATH"])
dev = torch.device("cuda")
x = torch.randn(16384, 60, 4, generator=torch.Generator().manual_seed(1)).to(dev)
m = x3.X3Model(SPEC, [{k: v.to(dev) for k, v in R.synthetic_params(SPEC, 1).items()}])
x3.mcd_batch(m, x, 10, seed=1, update_moving=False)
torch.cuda.synchronize()
lib.x3_prof_reset()
x3.mcd_batch(m, x, 20, seed=1, update_moving=False)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 128)()
lib.x3_prof_dump(buf)
for l in range(1, 6):
    v = [buf[l * 16 + i] for i in range(16)]
    nw, nl = max(v[4], 1), max(v[12], 1)
    tot = v[3] / nw
    print(f"layer {l}: MFMA waves {v[4]:5d}  cycles/wave {tot/1e6:7.2f}M  compute {v[0]/nw/tot*100:5.1f}%  "
          f"epilogue {v[1]/nw/tot*100:5.1f}%  barrier {v[2]/nw/tot*100:5.1f}%  staging-issue {v[5]/nw/tot*100:5.1f}%"
          + (f" | loaders {v[12]}: store {v[8]/nl/(v[11]/nl)*100:5.1f}% barrier {v[9]/nl/(v[11]/nl)*100:5.1f}% "
             f"load-issue {v[10]/nl/(v[11]/nl)*100:5.1f}%" if v[12] else ""))
