"""GPU numerics of the data-preparation kernels (csrc/prep.hip) vs fp64 NumPy references:
per-window standardisation (prepare_numpy_datasets.py:83-95) and SMOTE's exact k-NN search
(imblearn NearestNeighbors, prepare_numpy_datasets.py:185-187)."""
import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.data import balance, prepare
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext

pytestmark = pytest.mark.gpu


def _knn_ref(X, k):
    """Brute force: exact fp64 squared distances, (distance, index) order, self excluded."""
    n = X.shape[0]
    out = np.empty((n, k), dtype=np.int64)
    for i in range(n):
        d = ((X - X[i]) ** 2).sum(1)
        d[i] = np.inf
        out[i] = np.lexsort((np.arange(n), d))[:k]
    return out


def test_standardize_kernel_matches_numpy():
    _ext.require()
    rs = np.random.RandomState(3)
    x = rs.randn(3001, 60, 4) * rs.rand(1, 1, 4) * 50 + rs.randn(3001, 1, 4) * 10
    x[7, :, 2] = 4.0  # a flat channel: std 0 -> (x - mean) / 1e-8 == 0
    ref = (x - x.mean(1, keepdims=True)) / (x.std(1, keepdims=True) + 1e-8)
    got = torch.ops.apneauq.prep_standardize(torch.from_numpy(x).cuda(), 1e-8).cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)
    # the public entry point takes the HIP path on the GPU
    np.testing.assert_allclose(prepare.standardize_per_window(x, device="cuda"), ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("n,d,k", [(517, 240, 5), (1200, 240, 5), (300, 17, 12), (40, 240, 1)])
def test_knn_kernel_exact(n, d, k):
    _ext.require()
    rs = np.random.RandomState(n + d)
    X = rs.randn(n, d)
    X[5] = X[9]          # duplicate rows: equal distances, ties broken by index
    X[11] = X[9]
    X[20] = X[3] + 1e-9  # a near-tie
    got = torch.ops.apneauq.prep_knn(torch.from_numpy(X).cuda(), k).cpu().numpy()
    np.testing.assert_array_equal(got, _knn_ref(X, k))


def test_smote_hip_knn_matches_sklearn():
    _ext.require()
    rs = np.random.RandomState(2025)
    X = rs.randn(2400, 240)
    y = (rs.rand(2400) < 0.2).astype(np.int64)
    a = balance.SMOTE(random_state=2025, knn_device="hip").fit_resample(X, y)
    b = balance.SMOTE(random_state=2025, knn_device="sklearn").fit_resample(X, y)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_allclose(a[0], b[0], rtol=0, atol=0)


@pytest.mark.parametrize("n,d,k", [(300, 17, 20), (200, 400, 3)])
def test_knn_hip_route_falls_back_outside_kernel_range(n, d, k):
    """k > 16 or rows wider than the kernel's LDS tile: the 'hip' (and default) route must take the
    distance-GEMM path instead of raising from prep_knn."""
    assert not balance.hip_knn_supported(d, k)
    rs = np.random.RandomState(n)
    X = rs.randn(n, d)
    np.testing.assert_array_equal(balance.knn_indices(X, k, device="hip"), _knn_ref(X, k))
    np.testing.assert_array_equal(balance.knn_indices(X, k), _knn_ref(X, k))
