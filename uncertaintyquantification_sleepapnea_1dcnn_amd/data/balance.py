"""SMOTE over-sampling and random under-sampling (imbalanced-learn is not installed).

Algorithms and random streams follow imbalanced-learn 0.12 as used by
``prepare_numpy_datasets.py:180-220`` (``SMOTE(random_state=seed)``, k=5;
``RandomUnderSampler(random_state=seed)``), so a seed produces the same resampled set:

* SMOTE, per minority class with ``n = n_majority - n_class`` samples to create: k+1 nearest
  neighbours of every class sample within the class (self dropped); a fresh
  ``RandomState(seed)`` draws ``randint(0, n_class*k, n)`` (row = i // k, neighbour = i % k) then
  ``uniform(size=n)`` gaps; ``x_new = x[row] + gap * (x[nn] - x[row])``; synthetic rows are
  appended after the originals.
* RUS: one ``RandomState(seed)``; for every non-minority class (ascending label order)
  ``choice(n_class, n_minority, replace=False)``; minority kept whole; output grouped by class.

The k-NN search is the hot spot (O(n_class^2 * 240)); on a GPU it runs in the HIP kernel
``csrc/prep.hip:knn_kernel``: exact fp64 squared distances, per-thread register top-k,
(distance, index) order, self excluded.  ``device="torch"`` keeps the chunked distance-GEMM + ``topk``
formulation (CPU float64 or any torch device) as a reference path.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def _knn_numpy(X: np.ndarray, k: int) -> np.ndarray:
    from sklearn.neighbors import NearestNeighbors

    nn = NearestNeighbors(n_neighbors=k + 1).fit(X)
    return nn.kneighbors(X, return_distance=False)[:, 1:]


def _knn_torch(X: np.ndarray, k: int, device: str, chunk: int = 8192) -> np.ndarray:
    import torch

    A = torch.as_tensor(X, dtype=torch.float64 if device == "cpu" else torch.float32, device=device)
    sq = (A * A).sum(1)
    out = np.empty((A.shape[0], k), dtype=np.int64)
    cand = min(A.shape[0], k + 1 + 8)
    for s in range(0, A.shape[0], chunk):
        q = A[s: s + chunk]
        d = sq[s: s + chunk, None] + sq[None] - 2.0 * (q @ A.t())
        idx = torch.topk(d, cand, dim=1, largest=False).indices
        # exact re-rank of the candidate set (guards GEMM cancellation), stable on ties by index
        diff = A[idx] - q[:, None, :]
        ex = (diff.double() * diff.double()).sum(-1)
        self_pos = torch.arange(s, s + q.shape[0], device=A.device)[:, None]
        ex = torch.where(idx == self_pos, torch.full_like(ex, float("inf")), ex)  # drop the query itself
        # ascending exact distance, ties broken by index (as a sorted brute-force search)
        order = torch.argsort(ex * 0 + idx.double(), dim=1)
        idx, ex = torch.gather(idx, 1, order), torch.gather(ex, 1, order)
        order = torch.sort(ex, dim=1, stable=True).indices
        out[s: s + q.shape[0]] = torch.gather(idx, 1, order)[:, :k].cpu().numpy()
    return out


def _knn_hip(X: np.ndarray, k: int) -> np.ndarray:
    import torch

    from ..ops import _ext

    _ext.require()
    A = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float64)).to("cuda")
    return torch.ops.apneauq.prep_knn(A, int(k)).cpu().numpy()


def knn_indices(X: np.ndarray, k: int = 5, device: Optional[str] = None) -> np.ndarray:
    """k nearest neighbours of every row of X among the other rows, (distance, index) order.

    device: None (HIP kernel when a GPU is present, else scikit-learn), "hip", "sklearn", or a torch
    device string for the distance-GEMM reference path ("cpu", "cuda", or "torch" = the GPU)."""
    if device is None:
        try:
            import torch

            device = "hip" if torch.cuda.is_available() else "sklearn"
        except Exception:
            device = "sklearn"
    if device == "sklearn" or X.shape[0] <= k + 1:
        return _knn_numpy(X, k)
    if device in ("hip", "cuda") and hip_knn_supported(X.shape[1], k):
        return _knn_hip(X, k)
    # outside the kernel's range (k > 16 or rows too wide for its LDS tile) the distance-GEMM path
    return _knn_torch(X, k, "cuda" if device in ("torch", "hip") else device)


def hip_knn_supported(n_features: int, k: int) -> bool:
    """Range of the prep_knn kernel (csrc: top-k list of <= 16 in registers, a row tile of <= 320
    fp64 features in LDS)."""
    return k <= 16 and n_features <= 320


class SMOTE:
    def __init__(self, random_state: Optional[int] = None, k_neighbors: int = 5, n_jobs: Optional[int] = None,
                 knn_device: Optional[str] = None):
        self.random_state = random_state
        self.k_neighbors = k_neighbors
        self.knn_device = knn_device

    def fit_resample(self, X, y) -> Tuple[np.ndarray, np.ndarray]:
        X = np.asarray(X)
        y_in = y
        y = np.asarray(y)
        classes, counts = np.unique(y, return_counts=True)
        n_max = counts.max()
        Xs, ys = [X], [y]
        for cls, cnt in zip(classes, counts):
            n_new = int(n_max - cnt)
            if n_new == 0:
                continue
            Xc = X[y == cls]
            if Xc.shape[0] <= self.k_neighbors:
                raise ValueError(f"Expected n_neighbors <= n_samples_fit, got {self.k_neighbors + 1} > {Xc.shape[0]}")
            nns = knn_indices(Xc, self.k_neighbors, self.knn_device)
            rs = np.random.RandomState(self.random_state) if not isinstance(self.random_state, np.random.RandomState) \
                else self.random_state
            samples = rs.randint(low=0, high=nns.size, size=n_new)
            steps = 1.0 * rs.uniform(size=n_new)[:, None]
            rows = np.floor_divide(samples, nns.shape[1])
            cols = np.mod(samples, nns.shape[1])
            new = Xc[rows] + steps * (Xc[nns[rows, cols]] - Xc[rows])
            Xs.append(new.astype(X.dtype))
            ys.append(np.full(n_new, cls, dtype=y.dtype))
        Xr, yr = np.vstack(Xs), np.hstack(ys)
        if hasattr(y_in, "name") and hasattr(y_in, "values"):  # pandas Series in -> Series out (as imblearn)
            import pandas as pd

            yr = pd.Series(yr, name=y_in.name)
        return Xr, yr


class RandomUnderSampler:
    def __init__(self, random_state: Optional[int] = None, replacement: bool = False):
        self.random_state = random_state
        self.replacement = replacement

    def fit_resample(self, X, y):
        X = np.asarray(X)
        y_in = y
        y = np.asarray(y)
        classes, counts = np.unique(y, return_counts=True)
        n_min = counts.min()
        minority = classes[np.argmin(counts)]
        rs = np.random.RandomState(self.random_state)
        idx = np.empty(0, dtype=int)
        for cls in classes:
            cls_idx = np.flatnonzero(y == cls)
            if cls != minority:
                pick = rs.choice(range(np.count_nonzero(y == cls)), size=n_min, replace=self.replacement)
                cls_idx = cls_idx[pick]
            idx = np.concatenate((idx, cls_idx), axis=0)
        self.sample_indices_ = idx
        yr = y[idx]
        if hasattr(y_in, "name") and hasattr(y_in, "values"):
            import pandas as pd

            yr = pd.Series(yr, name=y_in.name)
        return X[idx], yr
