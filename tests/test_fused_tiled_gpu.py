"""GPU numerics of the fused multi-sample-tile kernels (``csrc/fused_tiled.hip``): the reference CNN
with MaxPool1D(2) after blocks 1-5 (/root/reference/models/train_deep_ensemble_cnns.py:36-66, pooling
lines) and on the north star's 30 s single-channel window.  Oracles: the CPU bf16 emulation of the same arithmetic (``generic.emulate``, fp32 last block), the
layer-wise HIP kernels (``csrc/generic_conv.hip``) and the fp32 reference model; dropout masks and
sharding invariance are checked bitwise."""
import dataclasses

import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC, ModelSpec
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, fused, generic

pytestmark = pytest.mark.gpu

POOLED = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                        for i, b in enumerate(DEFAULT_SPEC.blocks)))
SINGLE30 = ModelSpec(30, 1, DEFAULT_SPEC.blocks)
NETS = {"pooled": POOLED, "single30": SINGLE30}


def _setup(name, seed, n):
    _ext.require()
    spec = NETS[name]
    p = R.synthetic_params(spec, seed)
    x = torch.randn(n, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(seed + n))
    pk = generic.pack(spec, {k: v.cuda() for k, v in p.items()})
    assert "tiled_blob" in pk, f"{name} must take the fused kernel"
    return spec, p, x, pk


@pytest.mark.parametrize("name", list(NETS))
@pytest.mark.parametrize("n", [1, 3, 4, 7, 8, 9, 130])
def test_fused_tiled_deterministic(name, n):
    spec, p, x, pk = _setup(name, 3, n)
    out = generic.forward(pk, spec, x.to(torch.bfloat16).cuda(), n_pass=2, logits=True).cpu()
    assert torch.equal(out[0], out[1])
    emu = generic.emulate(spec, p, x, logits=True, last_fp32=True).reshape(-1)
    np.testing.assert_allclose(out[0].numpy(), emu.numpy(), atol=3e-3, rtol=3e-3)
    ref = R.forward(spec, p, x, return_logits=True).reshape(-1)
    np.testing.assert_allclose(out[0].numpy(), ref.numpy(), atol=5e-2, rtol=5e-2)


@pytest.mark.parametrize("name", list(NETS))
def test_fused_tiled_mc_dropout_masks_and_sharding(name):
    spec, p, x, pk = _setup(name, 4, 45)
    n, T = x.shape[0], 6
    xb = x.to(torch.bfloat16).cuda()
    out = generic.forward(pk, spec, xb, n_pass=T, dropout=True, seed=21, window_offset=300, logits=True).cpu()
    for t in range(T):
        emu = generic.emulate(spec, p, x, dropout=True, seed=21, pass_id=t, sample_ids=torch.arange(300, 300 + n),
                              logits=True, last_fp32=True)
        np.testing.assert_allclose(out[t].numpy(), emu.reshape(-1).numpy(), atol=5e-3, rtol=5e-3)
    # pass chunking and window sharding do not change a single bit (masks keyed by global ids)
    one = generic.forward(pk, spec, xb, n_pass=1, dropout=True, seed=21, pass_offset=4, window_offset=300,
                          logits=True).cpu()
    assert torch.equal(one[0], out[4])
    half = generic.forward(pk, spec, xb[17:], n_pass=T, dropout=True, seed=21, window_offset=317, logits=True).cpu()
    assert torch.equal(half, out[:, 17:])


@pytest.mark.parametrize("name", list(NETS))
def test_fused_tiled_matches_layerwise_kernels(name):
    """Cross-check against the layer-wise HIP path on the same model (bf16 activations between
    blocks there, fp32 last block here)."""
    spec, p, x, pk = _setup(name, 5, 96)
    lw = {k: v for k, v in pk.items() if k != "tiled_blob"}
    xb = x.to(torch.bfloat16).cuda()
    a = generic.forward(pk, spec, xb, n_pass=3, dropout=True, seed=9).cpu()
    b = generic.forward(lw, spec, xb, n_pass=3, dropout=True, seed=9).cpu()
    np.testing.assert_allclose(a.numpy(), b.numpy(), atol=5e-3)


@pytest.mark.parametrize("name", list(NETS))
def test_fused_tiled_members(name):
    """Deep-Ensemble layout: a (members, bytes) blob stack runs all members in one launch, each equal
    to its single-member launch."""
    _ext.require()
    spec = NETS[name]
    ps = [{k: v.cuda() for k, v in R.synthetic_params(spec, s).items()} for s in (11, 12, 13)]
    blobs = torch.stack([fused.pack_blob(spec, q) for q in ps])
    x = torch.randn(50, spec.input_length, spec.input_channels,
                    generator=torch.Generator().manual_seed(0)).to(torch.bfloat16).cuda()
    thr, dsc = fused.dropout_tables(spec)
    o = _ext.ops()
    launch = o.fused_pooled_forward if name == "pooled" else o.fused_single_forward
    allm = launch(x, blobs, 2, 0, 0, 7, True, False, thr, dsc).cpu()
    assert allm.shape == (3, 2, 50)
    for i in range(3):
        one = launch(x, blobs[i:i + 1].contiguous(), 2, 0, 0, 7, True, False, thr, dsc).cpu()
        assert torch.equal(one[0], allm[i])
