"""GPU numerics of the layer-wise HIP inference path for non-reference architectures
(``csrc/generic_conv.hip`` / ``ops/generic.py``): pooled blocks, the north-star
"30 s single-channel" window shape, odd filter counts.  Oracles: the CPU bf16 emulation of the same
arithmetic (tight) and the fp32 reference model (bf16 tolerance); dropout masks must match exactly."""
import dataclasses

import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC, BlockSpec, ModelSpec
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, fused, generic

pytestmark = pytest.mark.gpu

POOLED = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                        for i, b in enumerate(DEFAULT_SPEC.blocks)))
SINGLE30 = ModelSpec(30, 1, tuple(BlockSpec(f, k, r, pl) for f, k, r, pl in
                                  [(32, 7, 0.3, True), (48, 5, 0.3, False), (20, 3, 0.5, True)]))
ODD = ModelSpec(45, 3, tuple(BlockSpec(f, k, r) for f, k, r in [(36, 9, 0.2), (100, 1, 0.4), (12, 5, 0.1)]))
SPECS = {"pooled": POOLED, "single30": SINGLE30, "odd": ODD}


def _params(spec, seed):
    return R.synthetic_params(spec, seed)


@pytest.mark.parametrize("name", list(SPECS))
@pytest.mark.parametrize("n", [1, 7, 130])
def test_generic_deterministic(name, n):
    _ext.require()
    spec = SPECS[name]
    p = _params(spec, 5)
    x = torch.randn(n, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(n))
    pk = generic.pack(spec, {k: v.cuda() for k, v in p.items()})
    out = generic.forward(pk, spec, x.to(torch.bfloat16).cuda(), logits=True)[0].cpu()
    emu = generic.emulate(spec, p, x, logits=True).reshape(-1)
    ref = R.forward(spec, p, x, return_logits=True).reshape(-1)
    np.testing.assert_allclose(out.numpy(), emu.numpy(), atol=2e-2, rtol=2e-2)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=6e-2, rtol=6e-2)


@pytest.mark.parametrize("name", list(SPECS))
def test_generic_mc_dropout_masks(name):
    """Every pass's dropout masks are regenerated on the host: results match the emulation per pass,
    and chunking passes (pass_offset) does not change them."""
    _ext.require()
    spec = SPECS[name]
    p = _params(spec, 6)
    n, T = 40, 5
    x = torch.randn(n, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(1))
    pk = generic.pack(spec, {k: v.cuda() for k, v in p.items()})
    xb = x.to(torch.bfloat16).cuda()
    out = generic.forward(pk, spec, xb, n_pass=T, dropout=True, seed=11, window_offset=100).cpu()
    for t in range(T):
        emu = generic.emulate(spec, p, x, dropout=True, seed=11, pass_id=t, sample_ids=torch.arange(100, 100 + n))
        np.testing.assert_allclose(out[t].numpy(), emu.reshape(-1).numpy(), atol=1e-2, rtol=1e-2)
        one = generic.forward(pk, spec, xb, n_pass=1, dropout=True, seed=11, pass_offset=t, window_offset=100).cpu()
        np.testing.assert_array_equal(one[0].numpy(), out[t].numpy())
    # window sharding invariance: the second half on its own, with its global offset
    half = generic.forward(pk, spec, xb[n // 2:], n_pass=T, dropout=True, seed=11, window_offset=100 + n // 2).cpu()
    np.testing.assert_array_equal(half.numpy(), out[:, n // 2:].numpy())


def test_generic_matches_fused_on_reference_spec():
    """Cross-check of the two HIP paths on the architecture both implement."""
    _ext.require()
    p = {k: v.cuda() for k, v in _params(DEFAULT_SPEC, 7).items()}
    x = torch.randn(64, 60, 4, generator=torch.Generator().manual_seed(2)).to(torch.bfloat16).cuda()
    a = generic.forward(generic.pack(DEFAULT_SPEC, p), DEFAULT_SPEC, x, n_pass=3, dropout=True, seed=5).cpu()
    b = fused.fused_forward(x, fused.pack_blob(DEFAULT_SPEC, p), DEFAULT_SPEC, n_pass=3, dropout=True, seed=5)[0].cpu()
    np.testing.assert_allclose(a.numpy(), b.numpy(), atol=1e-2, rtol=1e-2)


def test_model_api_uses_generic_path():
    """mc_dropout_predict / deep_ensembles_predict / predict of a pooled bf16 model run on the HIP kernels
    (the fp32 default: tests/test_fp32_gpu.py)."""
    _ext.require()
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

    models = [AlarconCNN1D(spec=POOLED, seed=s, device="cuda", params=_params(POOLED, s), precision="bf16")
              for s in (1, 2)]
    assert all(m.uses_generic() and m.uses_hip() and not m.uses_fused() for m in models)
    x = np.random.default_rng(0).standard_normal((33, 60, 4)).astype(np.float32)
    mcd = U.mc_dropout_predict(models[0], x, n_pred=4, bn_mode="running", seed=3)
    assert mcd.shape == (4, 33, 1)
    p0 = {k: v.cpu() for k, v in models[0].store.as_dict().items()}
    for t in range(4):
        emu = generic.emulate(POOLED, p0, torch.from_numpy(x), dropout=True, seed=3, pass_id=t)
        np.testing.assert_allclose(mcd[t, :, 0], emu.reshape(-1).numpy(), atol=1e-2)
    de = U.deep_ensembles_predict(models, x)
    assert de.shape == (2, 33, 1)
    np.testing.assert_allclose(de[1], models[1].predict(x), atol=1e-6)
    ref = R.forward(POOLED, {k: v.cpu() for k, v in models[1].store.as_dict().items()}, torch.from_numpy(x))
    np.testing.assert_allclose(de[1], ref.numpy(), atol=2e-2)
