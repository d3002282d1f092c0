"""Golden NumPy implementations of the uncertainty metrics (SURVEY §4 test level 1).

Written from the math of ``uncertainty_quantification/uq_techniques.py:35-206`` (not copied):
per-window mean / ddof-0 variance over the T passes or M members, predictive entropy of the
mean H(E[p]) and expected entropy E[H(p)] in nats (SciPy ``entropy`` after clipping to
[1e-10, 1-1e-10]), mutual information max(H - E[H], 0), class-conditional mean variances,
bootstrap aggregates and percentile confidence intervals.  The HIP kernels
(``csrc/uq_reduce.hip``) are tested against these.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

AGG_KEYS = (
    "overall_mean_variance",
    "mean_variance_class_0",
    "mean_variance_class_1",
    "mean_total_pred_entropy",
    "mean_expected_aleatoric_entropy",
    "mean_mutual_info",
)


def binary_entropy_nats(p: np.ndarray, epsilon: float = 1e-10) -> np.ndarray:
    """H([1-p, p]) in nats with SciPy semantics: clip, renormalise, -sum x log x (dtype kept)."""
    p = np.asarray(p)
    q = 1 - p
    pc = np.clip(p, epsilon, 1 - epsilon)
    qc = np.clip(q, epsilon, 1 - epsilon)
    s = pc + qc
    pc, qc = pc / s, qc / s
    with np.errstate(divide="ignore", invalid="ignore"):
        h = -(np.where(pc > 0, pc * np.log(pc), 0) + np.where(qc > 0, qc * np.log(qc), 0))
    return h.astype(p.dtype if np.issubdtype(p.dtype, np.floating) else np.float64)


def binary_entropy_bits(p: np.ndarray, epsilon: float = 1e-9) -> np.ndarray:
    """Per-window CSV entropy of analyze_mcd_patient_level.py:109-115 (bits, +1e-9 inside log2)."""
    p = np.asarray(p)
    return -(p * np.log2(p + epsilon) + (1 - p) * np.log2(1 - p + epsilon))


def as_2d(predictions: np.ndarray) -> np.ndarray:
    """(T, N) / (T, N, 1) / (N,) -> (T, N)."""
    p = np.asarray(predictions)
    if p.ndim == 3 and p.shape[-1] == 1:
        p = p[..., 0]
    p = np.squeeze(p) if p.ndim > 2 else p
    if p.ndim == 1:
        p = p.reshape(1, -1)
    return p


def per_window(predictions: np.ndarray) -> Dict[str, np.ndarray]:
    p = as_2d(predictions)
    mean = np.mean(p, axis=0)
    var = np.var(p, axis=0)
    total = binary_entropy_nats(mean)
    expected = np.mean(np.stack([binary_entropy_nats(pt) for pt in p]), axis=0)
    mi = np.maximum(total - expected, 0)
    return {"mean_pred": mean, "pred_variance": var, "total_pred_entropy": total,
            "expected_aleatoric_entropy": expected, "mutual_info": mi}


def class_mean(values: np.ndarray, y: np.ndarray, cls: int) -> float:
    m = np.asarray(y) == cls
    return float(np.mean(values[m])) if np.any(m) else 0.0


def aggregates(w: Dict[str, np.ndarray], y: np.ndarray) -> Dict[str, float]:
    return {
        "overall_mean_variance": float(np.mean(w["pred_variance"])),
        "mean_variance_class_0": class_mean(w["pred_variance"], y, 0),
        "mean_variance_class_1": class_mean(w["pred_variance"], y, 1),
        "mean_total_pred_entropy": float(np.mean(w["total_pred_entropy"])),
        "mean_expected_aleatoric_entropy": float(np.mean(w["expected_aleatoric_entropy"])),
        "mean_mutual_info": float(np.mean(w["mutual_info"])),
    }


def parity_bootstrap_indices(n: int, n_bootstrap: int, random_state: Optional[int]) -> np.ndarray:
    """Indices drawn exactly like the reference: global-seeded legacy ``np.random.choice``.

    ``uq_techniques.py:130-142`` reseeds the global RandomState and draws
    ``np.random.choice(n, n, replace=True)`` per iteration; a private RandomState with the same
    seed produces the same stream without touching global state.
    """
    rs = np.random.RandomState(random_state) if random_state is not None else np.random.mtrand._rand
    return np.stack([rs.choice(n, n, replace=True) for _ in range(n_bootstrap)]) if n_bootstrap else np.zeros((0, n), int)


def bootstrap_from_windows(w: Dict[str, np.ndarray], y: np.ndarray, idx: np.ndarray) -> List[Dict[str, float]]:
    """Bootstrap aggregates by gathering the (resampling-invariant) per-window metrics."""
    out = []
    y = np.asarray(y)
    for ix in idx:
        out.append(aggregates({k: v[ix] for k, v in w.items()}, y[ix]))
    return out


def confidence_intervals(results: List[Dict[str, float]], alpha: float = 0.05) -> Dict[str, float]:
    ci: Dict[str, float] = {}
    if not results:
        return ci
    for k in results[0].keys():
        vals = [r[k] for r in results]
        ci[f"{k}_mean"] = float(np.mean(vals))
        ci[f"{k}_ci_lower"] = float(np.percentile(vals, 100 * alpha / 2))
        ci[f"{k}_ci_upper"] = float(np.percentile(vals, 100 * (1 - alpha / 2)))
    return ci
