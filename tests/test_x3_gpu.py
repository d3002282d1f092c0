"""GPU numerics of the fp32-faithful (fp16x3 MFMA) layer-wise inference engine (ops/x3.py,
csrc/x3_layers.hip) against the fp32 PyTorch reference model (models/reference.py), on the same
weights, inputs and counter-based dropout masks.

Bound (VERDICT r2 "next round" item 1): max |dp| <= 1e-5 per window for batch-BN MC Dropout (the
reference's model(x, training=True), uq_techniques.py:22), standard MC Dropout and Deep-Ensemble
predict (uq_techniques.py:29).  The fp64 evaluation of the same model is reported as the exact oracle:
the engine must be as close to it as the fp32 reference is (both differ from it by fp32 rounding)."""
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, x3

pytestmark = pytest.mark.gpu

BOUND = 1e-5


def _params(seed, dev):
    return {k: v.to(dev) for k, v in R.synthetic_params(SPEC, seed).items()}


def _ref(p, x, dtype=None, **kw):
    """Reference forward on the CPU (fp32 by default, float64 oracle with dtype=torch.float64)."""
    pc = {k: v.detach().cpu().to(dtype or torch.float32).clone() for k, v in p.items()}
    return R.forward(SPEC, pc, x.detach().cpu(), dtype=dtype, **kw).reshape(-1), pc


def _x(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 60, 4, generator=g)


@pytest.mark.parametrize("n", [37, 256])
def test_de_running_bn_matches_fp32_reference(n):
    _ext.require()
    dev = torch.device("cuda")
    ps = [_params(100 + m, dev) for m in range(3)]
    model = x3.X3Model(SPEC, ps)
    x = _x(n, n)
    p = x3.forward_running(model, x.to(dev))  # (3, 1, n)
    assert p.shape == (3, 1, n)
    for m in range(3):
        r32, _ = _ref(ps[m], x)
        r64, _ = _ref(ps[m], x, dtype=torch.float64)
        d = (p[m, 0].cpu() - r32).abs().max().item()
        d64 = (p[m, 0].cpu().double() - r64).abs().max().item()
        ref_err = (r32.double() - r64).abs().max().item()
        assert d <= BOUND, f"member {m}: max |dp| vs fp32 reference {d:.3e}"
        assert d64 <= max(4 * ref_err, 2e-6), f"member {m}: vs fp64 {d64:.3e} (fp32 reference itself {ref_err:.3e})"


def test_de_logits_match():
    _ext.require()
    dev = torch.device("cuda")
    ps = [_params(7, dev)]
    model = x3.X3Model(SPEC, ps)
    x = _x(64, 3)
    lg = x3.forward_running(model, x.to(dev), logits=True)[0, 0].cpu()
    r, _ = _ref(ps[0], x, return_logits=True)
    assert (lg - r).abs().max().item() <= 4e-5 * max(1.0, r.abs().max().item())


@pytest.mark.parametrize("n,T", [(37, 3), (130, 2)])
def test_mcd_running_bn_matches_fp32_reference(n, T):
    _ext.require()
    dev = torch.device("cuda")
    p = _params(11, dev)
    model = x3.X3Model(SPEC, [p])
    x = _x(n, 5)
    seed, base, off = 77, 1234, 500
    ph = x3.forward_running(model, x.to(dev), n_pass=T, dropout=True, seed=seed, pass_offset=base, window_offset=off)
    assert ph.shape == (1, T, n)
    ids = torch.arange(off, off + n)
    for t in range(T):
        r, _ = _ref(p, x, dropout=True, bn_batch_stats=False, seed=seed, pass_id=base + t, sample_ids=ids)
        d = (ph[0, t].cpu() - r).abs().max().item()
        assert d <= BOUND, f"pass {t}: max |dp| {d:.3e}"


@pytest.mark.parametrize("n,T", [(37, 3), (256, 2)])
def test_mcd_batch_bn_matches_fp32_reference(n, T):
    """Reference semantics: model(x, training=True) T times (batch moments over all n windows per pass,
    dropout, moving averages updated once per pass and per layer)."""
    _ext.require()
    dev = torch.device("cuda")
    p = _params(13, dev)
    model = x3.X3Model(SPEC, [p])
    x = _x(n, 9)
    seed, base = 2025, 40
    ph = x3.mcd_batch(model, x.to(dev), T, seed=seed, pass_base=base, update_moving=True)
    assert ph.shape == (T, n)
    pc = {k: v.detach().cpu().clone() for k, v in _params(13, "cpu").items()}
    ids = torch.arange(n)
    worst = 0.0
    for t in range(T):
        r = R.forward(SPEC, pc, x, dropout=True, bn_batch_stats=True, update_moving=True, seed=seed, pass_id=base + t,
                      sample_ids=ids).reshape(-1)
        worst = max(worst, (ph[t].cpu() - r).abs().max().item())
    assert worst <= BOUND, f"max |dp| {worst:.3e}"
    # the moving-average side effect (p's tensors are views updated in place by the engine)
    for i in range(1, 7):
        for nme in ("moving_mean", "moving_variance"):
            k = f"batchnorm_{i}/{nme}"
            torch.testing.assert_close(p[k].cpu(), pc[k], atol=2e-6, rtol=2e-6)


def test_mcd_batch_chunked_equals_unchunked():
    _ext.require()
    dev = torch.device("cuda")
    x = _x(41, 2).to(dev)
    outs = []
    for ms in (None, 41 * 2):  # all passes in one chunk / two passes per chunk
        model = x3.X3Model(SPEC, [_params(3, dev)])
        outs.append(x3.mcd_batch(model, x, 5, seed=1, update_moving=False, max_samples=ms))
    torch.testing.assert_close(outs[0], outs[1], atol=2e-6, rtol=0)


def test_mcd_batch_window_chunked_equals_one_shot():
    """More windows than fit at one pass (VERDICT r2 missing #4): the two-phase window-chunked schedule
    (moments of block l over window chunks, blocks below recomputed) gives the one-shot result."""
    _ext.require()
    dev = torch.device("cuda")
    x = _x(41, 4).to(dev)
    res = []
    for ms in (None, 16):  # one shot / chunks of 16, 16, 9 windows
        p = _params(5, dev)
        model = x3.X3Model(SPEC, [p])
        ph = x3.mcd_batch(model, x, 3, seed=9, pass_base=2, window_offset=100, update_moving=True, max_samples=ms)
        res.append((ph, {k: v.clone() for k, v in p.items() if "moving" in k}))
    torch.testing.assert_close(res[1][0], res[0][0], atol=1e-6, rtol=0)
    for k in res[0][1]:
        torch.testing.assert_close(res[1][1][k], res[0][1][k], atol=1e-6, rtol=1e-6)
