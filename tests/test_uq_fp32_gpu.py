"""The user-facing inference entry points run the fp32-faithful engine by default (the reference
computes in fp32, Keras defaults): ``model.predict`` / ``model(x)`` (uq_techniques.py:29's
``m.predict``), MC Dropout with batch statistics (``model(x, training=True)`` x T, uq_techniques.py:22)
and with running statistics, and Deep-Ensemble predict -- each within 1e-5 of the fp32 reference model
on the same weights and counter-based masks.  ``precision="bf16"`` selects the bf16 kernels."""
import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext
from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

pytestmark = pytest.mark.gpu
BOUND = 1e-5


def _x(n=96, seed=3):
    return torch.randn(n, 60, 4, generator=torch.Generator().manual_seed(seed))


def _cpu_params(m):
    return {k: v.detach().cpu().clone() for k, v in m.store.as_dict().items()}


def test_predict_uses_fp32_engine():
    _ext.require()
    m = AlarconCNN1D(seed=4, device="cuda")
    assert m.precision == "fp32" and m.uses_x3()
    x = _x()
    got = m.predict(x.numpy())[:, 0]
    ref = torch.sigmoid(R.forward(m.spec, _cpu_params(m), x, return_logits=True)).reshape(-1).numpy()
    assert np.abs(got - ref).max() <= BOUND
    b = AlarconCNN1D(seed=4, device="cuda", precision="bf16")
    assert not b.uses_x3()
    gb = b.predict(x.numpy())[:, 0]
    assert np.abs(gb - ref).max() > np.abs(got - ref).max()  # the bf16 kernels really ran


@pytest.mark.parametrize("bn_mode", ["batch", "running"])
def test_mc_dropout_predict_fp32(bn_mode):
    _ext.require()
    m = AlarconCNN1D(seed=6, device="cuda")
    p0 = _cpu_params(m)
    x = _x(70, 5)
    T = 3
    got = U.mc_dropout_predict(m, x.numpy(), n_pred=T, bn_mode=bn_mode, seed=21, distributed=False)[..., 0]
    ids = torch.arange(70)
    for t in range(T):
        r = torch.sigmoid(R.forward(m.spec, p0, x, dropout=True, bn_batch_stats=(bn_mode == "batch"),
                                    update_moving=(bn_mode == "batch"), seed=21, pass_id=t, sample_ids=ids,
                                    return_logits=True)).reshape(-1).numpy()
        assert np.abs(got[t] - r).max() <= BOUND, f"pass {t}"
    if bn_mode == "batch":  # the moving-average side effect reached the model (and p0 holds the CPU replay)
        for k, v in _cpu_params(m).items():
            if "moving" in k:
                torch.testing.assert_close(v, p0[k], atol=2e-6, rtol=2e-6)


def test_deep_ensembles_predict_fp32():
    _ext.require()
    ms = [AlarconCNN1D(seed=30 + i, device="cuda") for i in range(3)]
    x = _x(50, 8)
    got = U.deep_ensembles_predict(ms, x.numpy(), distributed=False)[..., 0]
    for i, m in enumerate(ms):
        r = torch.sigmoid(R.forward(m.spec, _cpu_params(m), x, return_logits=True)).reshape(-1).numpy()
        assert np.abs(got[i] - r).max() <= BOUND
