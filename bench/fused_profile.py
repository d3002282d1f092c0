"""Launch the fused MCD kernel a few times (target for rocprofv3 counter collection)."""
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as S
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused

x = torch.randn(16384, 60, 4, device="cuda").to(torch.bfloat16)
blob = fused.pack_blob(S, {k: v.cuda() for k, v in R.init_params(S, 1).items()}).unsqueeze(0)
for _ in range(3):
    fused.fused_forward(x, blob, S, n_pass=50, dropout=True, seed=7)
torch.cuda.synchronize()
