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


@pytest.mark.parametrize("sign", ["", "1,2,3,4"])
@pytest.mark.parametrize("bn", ["batch", "running"])
def test_mask_side_matches_reference(monkeypatch, sign, bn):
    """Every block's dropout mask drawn by the consumer's staging (hash) or by the producer's epilogue (R's
    sign bit; ops/x3.py _SIGN_DEFAULT picks per layer): both are the reference's masks."""
    _ext.require()
    monkeypatch.setenv("APNEAUQ_X3_SIGN_MASK", sign)
    dev = torch.device("cuda")
    x = _x(45, 4)
    p = _params(17, dev)
    pc = {k: v.detach().cpu().clone() for k, v in p.items()}
    model = x3.X3Model(SPEC, [p])
    ids = torch.arange(45)
    if bn == "batch":
        ph = x3.mcd_batch(model, x.to(dev), 2, seed=8, pass_base=3, update_moving=False)
    else:
        ph = x3.forward_running(model, x.to(dev), n_pass=2, dropout=True, seed=8, pass_offset=3)[0]
    for t in range(2):
        r = R.forward(SPEC, pc, x, dropout=True, bn_batch_stats=bn == "batch", seed=8, pass_id=3 + t,
                      sample_ids=ids).reshape(-1)
        assert (ph[t].cpu() - r).abs().max().item() <= BOUND


def test_de_chunking_and_float64_large():
    """the Deep-Ensemble path picks its fp16 prescale per member and block from the whole
    launch's sums of squares (ops/x3.py _predict_members), so a window's last bits may depend on the
    windows sharing its chunk.  At 4096 windows (bound overshoot ~2^9 of a window's own maximum) the
    window-chunked result (8 chunks) stays within 1e-6 of the one-launch result, and both within the
    usual bounds of the fp32 reference and the float64 oracle."""
    _ext.require()
    dev = torch.device("cuda")
    n = 4096
    ps = [_params(300 + m, dev) for m in range(2)]
    model = x3.X3Model(SPEC, ps)
    x = _x(n, 99)
    one = x3.forward_running(model, x.to(dev))
    chunked = x3.forward_running(model, x.to(dev), max_samples=2 * (n // 8))
    assert one.shape == chunked.shape == (2, 1, n)
    assert (one - chunked).abs().max().item() <= 1e-6
    for m in range(2):
        r32, _ = _ref(ps[m], x)
        r64, _ = _ref(ps[m], x, dtype=torch.float64)
        ref_err = (r32.double() - r64).abs().max().item()
        for got in (one, chunked):
            assert (got[m, 0].cpu() - r32).abs().max().item() <= BOUND
            assert (got[m, 0].cpu().double() - r64).abs().max().item() <= max(4 * ref_err, 2e-6)


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


def _scaled_params(seed, dev, case, dense=None):
    """Weights whose BN affines put every split activation far outside the fp16 comfort range:
    "huge": |a| ~ 1e4 (up to ~1e5 with the dropout rescale, beyond fp16's 65504); "tiny": |a| ~ 1e-6
    (below fp16's 6e-5 normal range, where the lo half would be lost).  Conv biases / moving stats are
    chosen so that every block keeps that scale, and the dense kernel brings the logits back to O(1)."""
    p = _params(seed, dev)
    for i in range(1, 7):
        g, mv = p[f"batchnorm_{i}/gamma"], p[f"batchnorm_{i}/moving_variance"]
        p[f"batchnorm_{i}/moving_mean"].zero_()
        if case == "huge":
            g.fill_(1e4)
            mv.fill_(1.0 if i == 1 else 1e8)  # running BN: R_l ~ 1e4 -> a_l ~ 1e4
        else:
            g.fill_(1e-6 if i == 1 else SPEC.bn_epsilon ** 0.5)  # a_1 ~ 1e-6; then a_l ~ R_l ~ 1e-6
            mv.fill_(1.0 if i == 1 else 0.0)
            p[f"batchnorm_{i}/beta"].zero_()
            p[f"conv1d_{i}/bias"].zero_()
    p["output_layer/kernel"].mul_(dense or (1e-4 if case == "huge" else 1e6))
    return p


@pytest.mark.parametrize("case", ["huge", "tiny"])
def test_range_safe_activation_split(case):
    """the fp16 hi/lo split of each block's input is prescaled by a power of two
    derived from the tracked channel maxima of the block's ReLU output (ops/x3.py, x3_aff), so BN
    gamma = 1e4 and 1e-6-scale activations keep the fp32-faithful precision: Deep-Ensemble logits within
    1e-5 relative, batch-BN MC Dropout within the usual 1e-5 |dp|."""
    _ext.require()
    dev = torch.device("cuda")
    x = _x(48, 21)
    p = _scaled_params(31, dev, case)
    model = x3.X3Model(SPEC, [p])
    lg = x3.forward_running(model, x.to(dev), logits=True)[0, 0].cpu()
    r, _ = _ref(p, x, return_logits=True)
    assert torch.isfinite(lg).all()
    rel = ((lg - r).abs() / r.abs().clamp_min(1e-3)).max().item()
    assert rel <= 1e-5, f"{case}: DE logits max relative error {rel:.3e}"
    # batch BN centres each channel: the tiny case's dense kernel is 10x larger to keep the logits O(1)
    pb = _scaled_params(31, dev, case, dense=1e7 if case == "tiny" else None)
    pc = {k: v.detach().cpu().clone() for k, v in pb.items()}
    ph = x3.mcd_batch(x3.X3Model(SPEC, [pb]), x.to(dev), 2, seed=3, pass_base=0, update_moving=False)
    ids = torch.arange(x.shape[0])
    for t in range(2):
        ref = R.forward(SPEC, pc, x, dropout=True, bn_batch_stats=True, update_moving=False, seed=3, pass_id=t,
                        sample_ids=ids).reshape(-1)
        d = (ph[t].cpu() - ref).abs().max().item()
        assert d <= BOUND, f"{case}: batch-BN MC Dropout pass {t}: max |dp| {d:.3e}"
        assert 0.02 < ref.std().item(), "the logits must not be saturated (the test would be vacuous)"
