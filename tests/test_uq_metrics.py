"""UQ metric parity: framework API vs an independent re-statement of the reference algorithm
(uq_techniques.py:40-206: full metric recomputation on every bootstrap resample, global-seeded
legacy RNG).  Also covers the bootstrap gather reformulation and the CI keys."""
import os

import numpy as np
import pytest
from scipy.stats import entropy

from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import metrics as M
from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U


def _ref_dist(preds, y):
    p = np.squeeze(preds)
    if p.ndim == 1:
        p = p.reshape(1, -1)
    mean = p.mean(0)
    var = p.var(0)
    H = lambda q: entropy(np.clip(np.stack([1 - q, q], -1), 1e-10, 1 - 1e-10), axis=1)
    tot = H(mean)
    exp = np.mean([H(r) for r in p], axis=0)
    mi = np.maximum(tot - exp, 0)
    c0, c1 = y == 0, y == 1
    return dict(mean_pred=mean, pred_variance=var, total_pred_entropy=tot, expected_aleatoric_entropy=exp,
                mutual_info=mi, overall_mean_variance=var.mean(),
                mean_variance_class_0=var[c0].mean() if c0.any() else 0.0,
                mean_variance_class_1=var[c1].mean() if c1.any() else 0.0)


def _ref_bootstrap(preds, y, B, seed):
    np.random.seed(seed)
    n = preds.shape[1]
    out = []
    for _ in range(B):
        idx = np.random.choice(n, n, replace=True)
        d = _ref_dist(preds[:, idx], y[idx])
        out.append({"overall_mean_variance": d["overall_mean_variance"],
                    "mean_variance_class_0": d["mean_variance_class_0"],
                    "mean_variance_class_1": d["mean_variance_class_1"],
                    "mean_total_pred_entropy": np.mean(d["total_pred_entropy"]),
                    "mean_expected_aleatoric_entropy": np.mean(d["expected_aleatoric_entropy"]),
                    "mean_mutual_info": np.mean(d["mutual_info"])})
    return out


@pytest.fixture
def data():
    rs = np.random.RandomState(7)
    T, N = 9, 400
    p = np.clip(rs.rand(T, N) * 0.9 + rs.randn(T, N) * 0.05, 0, 1).astype(np.float32)
    p[0, :5] = 0.0
    p[1, 5:10] = 1.0
    y = (rs.rand(N) > 0.6).astype(int)
    return p, y


def test_per_window_matches_reference(data):
    p, y = data
    ref = _ref_dist(p, y)
    got = U.uq_evaluation_dist(p, y)
    assert set(got) == set(ref)
    for k in ref:
        np.testing.assert_allclose(np.asarray(got[k], np.float64), np.asarray(ref[k], np.float64), rtol=2e-5, atol=2e-6,
                                   err_msg=k)


def test_bootstrap_gather_equals_recompute(data):
    p, y = data
    ref = _ref_bootstrap(p, y, 12, 2025)
    got = U.bootstrap_metrics(p, y, 12, 2025, device="cpu")
    assert len(got) == 12
    for r, g in zip(ref, got):
        for k in r:
            assert g[k] == pytest.approx(float(r[k]), rel=3e-5, abs=1e-7), k


def test_confidence_interval_keys(data):
    p, y = data
    res = U.evaluate_uq_methods(p[:, :, None], y, "t", n_bootstrap=8, random_state=1, make_plots=False)
    assert len(res) == 24
    for k in M.AGG_KEYS:
        assert {f"{k}_mean", f"{k}_ci_lower", f"{k}_ci_upper", k} <= set(res)
        assert res[f"{k}_ci_lower"] <= res[f"{k}_ci_upper"]


def test_entropy_units():
    p = np.array([0.0, 0.5, 1.0, 0.25], np.float32)
    nats = M.binary_entropy_nats(p)
    assert nats[1] == pytest.approx(np.log(2), rel=1e-6)
    bits = M.binary_entropy_bits(p)
    assert bits[1] == pytest.approx(1.0, rel=1e-6)
    np.testing.assert_allclose(U.safe_entropy(np.stack([1 - p, p], -1), axis=1), nats, rtol=1e-5, atol=1e-7)


def test_eager_device_formulas_match_numpy(data):
    import torch
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import uq as uq_ops

    p, y = data
    m = uq_ops.metrics(torch.from_numpy(p)).numpy()
    w = M.per_window(p)
    np.testing.assert_allclose(m[uq_ops.VAR], w["pred_variance"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(m[uq_ops.ENT_NATS], w["total_pred_entropy"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(m[uq_ops.MI], w["mutual_info"], rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(m[uq_ops.ENT_BITS], M.binary_entropy_bits(w["mean_pred"]), rtol=1e-5, atol=1e-6)
    idx = M.parity_bootstrap_indices(p.shape[1], 5, 3)
    b = uq_ops.bootstrap(torch.from_numpy(m), torch.from_numpy(y), 5, idx=torch.from_numpy(idx)).numpy()
    ref = M.bootstrap_from_windows(w, y, idx)
    for i in range(5):
        np.testing.assert_allclose(b[i], [ref[i][k] for k in M.AGG_KEYS], rtol=1e-4, atol=1e-7)


def test_plots_and_demo(tmp_path, data):
    p, y = data
    out = tmp_path / "plots"
    U.evaluate_uq_methods(p[:, :, None], y, "lbl", n_bootstrap=4, random_state=0, output_plot_dir=str(out))
    names = sorted(os.listdir(out))
    assert any(n.startswith("hist_") for n in names) and any(n.startswith("bar_class_variance") for n in names)
    U.plot_uncertainty_metric(p.var(0), "lbl", "variance", output_dir=str(out))
    assert any(n.startswith("line_") for n in os.listdir(out))
    res = U.demo(output_plot_dir=str(tmp_path / "demo"), n_samples=200)
    assert res is not None and len(res) == 24
