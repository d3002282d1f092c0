"""GPU numerics of the fused whole-network kernel vs the CPU fp32 reference and bf16 emulation."""
import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as S
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused as F

pytestmark = pytest.mark.gpu


def _params(seed):
    p = R.init_params(S, seed)
    g = torch.Generator().manual_seed(seed + 100)
    for i, b in enumerate(S.blocks, start=1):
        c = b.filters
        p[f"batchnorm_{i}/moving_mean"] = torch.rand(c, generator=g) * 0.5
        p[f"batchnorm_{i}/moving_variance"] = torch.rand(c, generator=g) + 0.5
        p[f"batchnorm_{i}/gamma"] = torch.rand(c, generator=g) + 0.5
        p[f"batchnorm_{i}/beta"] = torch.randn(c, generator=g) * 0.1
        p[f"conv1d_{i}/bias"] = torch.randn(c, generator=g) * 0.05
    return p


def test_layout_matches_kernel():
    _ext.require()
    F.check_layout()


@pytest.mark.parametrize("n", [1, 2, 37])
def test_fused_deterministic_matches_reference(n):
    _ext.require()
    p = _params(3)
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, 60, 4, generator=g)
    blob = F.pack_blob(S, p).cuda()
    xb = x.to(torch.bfloat16).cuda()
    out = F.fused_forward(xb, blob, S, logits=True)[0, 0].cpu()
    emu = F.emulate_blob_forward(blob, x, logits=True)
    ref = R.forward(S, p, x, dropout=False, bn_batch_stats=False, return_logits=True).reshape(-1)
    assert torch.allclose(out, emu, atol=2e-2, rtol=2e-2), (out - emu).abs().max()
    assert torch.allclose(out, ref, atol=6e-2, rtol=5e-2), (out - ref).abs().max()


def test_fused_mc_dropout_masks_match_host():
    _ext.require()
    p = _params(4)
    n, T, seed = 9, 3, 1234
    x = torch.randn(n, 60, 4, generator=torch.Generator().manual_seed(1))
    blob = F.pack_blob(S, p).cuda()
    out = F.fused_forward(x.to(torch.bfloat16).cuda(), blob, S, n_pass=T, dropout=True, seed=seed, logits=True)[0].cpu()
    for t in range(T):
        emu = F.emulate_blob_forward(blob, x, dropout=True, seed=seed, pass_id=t, logits=True)
        assert torch.allclose(out[t], emu, atol=3e-2, rtol=3e-2), (t, (out[t] - emu).abs().max())
    assert (out[0] - out[1]).abs().max() > 1e-3  # passes differ


def test_fused_sharding_invariance():
    _ext.require()
    p = _params(5)
    n, T, seed = 20, 2, 99
    x = torch.randn(n, 60, 4, generator=torch.Generator().manual_seed(2)).to(torch.bfloat16).cuda()
    blob = F.pack_blob(S, p).cuda()
    full = F.fused_forward(x, blob, S, n_pass=T, dropout=True, seed=seed)[0]
    a = F.fused_forward(x[:7].contiguous(), blob, S, n_pass=T, dropout=True, seed=seed, window_offset=0)[0]
    b = F.fused_forward(x[7:].contiguous(), blob, S, n_pass=T, dropout=True, seed=seed, window_offset=7)[0]
    assert torch.equal(torch.cat([a, b], dim=1), full)


def test_fused_multi_member():
    _ext.require()
    ps = [_params(10 + m) for m in range(3)]
    x = torch.randn(11, 60, 4, generator=torch.Generator().manual_seed(3))
    blobs = torch.stack([F.pack_blob(S, p) for p in ps]).cuda()
    out = F.fused_forward(x.to(torch.bfloat16).cuda(), blobs, S)[:, 0].cpu()
    for m, p in enumerate(ps):
        ref = R.forward(S, p, x, dropout=False, bn_batch_stats=False).reshape(-1)
        assert torch.allclose(out[m], ref, atol=1e-2), (m, (out[m] - ref).abs().max())


def test_fused_bitwise_deterministic_and_pass_offset():
    """Same seed => bitwise-identical MC-Dropout outputs across runs; a pass-sharded run
    (pass_offset) reproduces the corresponding rows of the full run (SURVEY §5 determinism)."""
    _ext.require()
    p = _params(6)
    x = torch.randn(300, 60, 4, generator=torch.Generator().manual_seed(4)).to(torch.bfloat16).cuda()
    blob = F.pack_blob(S, p).cuda()
    a = F.fused_forward(x, blob, S, n_pass=8, dropout=True, seed=5)[0]
    b = F.fused_forward(x, blob, S, n_pass=8, dropout=True, seed=5)[0]
    assert torch.equal(a, b)
    tail = F.fused_forward(x, blob, S, n_pass=3, dropout=True, seed=5, pass_offset=5)[0]
    assert torch.equal(tail, a[5:])
    c = F.fused_forward(x, blob, S, n_pass=8, dropout=True, seed=6)[0]
    assert not torch.equal(a, c)


@pytest.mark.parametrize("limit", [1000, 250])
def test_fused_chunked_launches_equal_one_launch(monkeypatch, limit):
    """Calls with n_pass * N >= 2^31 samples are split into pass (and window) chunks; with the
    per-launch limit lowered, the chunked result is bitwise that of one launch (global mask keys)."""
    _ext.require()
    ps = [_params(20 + m) for m in range(2)]
    x = torch.randn(300, 60, 4, generator=torch.Generator().manual_seed(8)).to(torch.bfloat16).cuda()
    blobs = torch.stack([F.pack_blob(S, p) for p in ps]).cuda()
    full = F.fused_forward(x, blobs, S, n_pass=7, dropout=True, seed=11, pass_offset=3, window_offset=5)
    monkeypatch.setattr(F, "_MAX_SAMPLES", limit)
    chunked = F.fused_forward(x, blobs, S, n_pass=7, dropout=True, seed=11, pass_offset=3, window_offset=5)
    assert chunked.shape == full.shape and torch.equal(chunked, full)
