"""Drop-in equivalent of the reference's ``uncertainty_quantification/uq_techniques.py`` API.

Same function names, signatures, return shapes and dictionary keys as the reference
(``uq_techniques.py:12-391``), executed MI355X-first:

* :func:`mc_dropout_predict` runs all ``n_pred`` stochastic passes in ONE fused HIP launch
  (``bn_mode="running"``, standard MC Dropout) or reproduces the reference exactly
  (``bn_mode="batch"``: every pass is ``model(x, training=True)`` — dropout on, BatchNorm on the
  statistics of the whole test set, moving averages updated);
* :func:`deep_ensembles_predict` runs every member in one fused launch (inference BN, no dropout);
* :func:`uq_evaluation_dist`, :func:`bootstrap_metrics` and :func:`evaluate_uq_methods` compute the
  per-window metrics with the HIP ``uq_reduce`` kernel and the B bootstrap replicates with the
  gather-reduce kernel when the data is on (or the machine has) a GPU, else with NumPy.  Bootstrap
  indices are drawn with the reference's legacy ``RandomState.choice`` stream (parity) unless
  ``parity=False`` (device counter-hash indices).

Wall-clock prints mirror the reference (``uq_techniques.py:23,31,347``).
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional

import numpy as np
from scipy.stats import entropy

from . import metrics as M

try:  # plotting is optional (headless Agg backend)
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
except Exception:  # pragma: no cover
    plt = None


def _torch():
    import torch

    return torch


def _gpu_ok() -> bool:
    torch = _torch()
    if not torch.cuda.is_available():
        return False
    from ..ops import _ext

    return _ext.available()


# ===================== Core Prediction Functions =====================
def mc_dropout_predict(model, x_test_data, n_pred: int = 50, bn_mode: str = "batch", seed: Optional[int] = None,
                       as_numpy: bool = True, distributed: Optional[bool] = None):
    """MC Dropout predictions (n_pred, samples, 1) float32.

    ``bn_mode="batch"`` (default, reference parity): each pass is ``model(x, training=True)``.
    ``bn_mode="running"``: dropout on, BatchNorm on running statistics — all passes in one fused
    kernel launch on the GPU.  Under ``torchrun`` (``distributed=None`` = auto) the windows are
    sharded over the ranks and the result is all-gathered (``uq/distributed.py``).
    """
    torch = _torch()
    start_time = time.time()
    if bn_mode not in ("batch", "running"):
        raise ValueError("bn_mode must be 'batch' or 'running'")
    from . import distributed as D

    if (D.active() if distributed is None else distributed):
        out = D.mc_dropout_predict_sharded(model, x_test_data, n_pred, bn_mode, seed)
    elif bn_mode == "running" and getattr(model, "uses_hip", lambda: False)():
        # fused whole-network kernel (reference architecture) or the layer-wise HIP kernels (any spec);
        # like model(x, training=True), every call draws fresh masks (pass ids advance per call)
        x = model._as_input(x_test_data)
        base = model._call_counter
        out = model.hip_infer(x, n_pass=n_pred, dropout=True, seed=seed, pass_offset=base).unsqueeze(-1)
        model._call_counter = base + n_pred
    elif bn_mode == "running":
        x = model._as_input(x_test_data)
        base = model._call_counter
        out = torch.stack([torch.sigmoid(model.logits(x, dropout=True, bn_batch_stats=False, pass_id=base + t,
                                                      seed=seed)) for t in range(n_pred)])
        model._call_counter = base + n_pred
    else:
        from ..ops import bn_batch

        out = bn_batch.mc_dropout_batch_bn(model, x_test_data, n_pred, seed=seed)
    if as_numpy:
        out = out.float().cpu().numpy()
    print(f"MC Dropout completed in {time.time() - start_time:.1f}s ({n_pred} passes)")
    return out


def deep_ensembles_predict(ensemble_models: List, x_test_data, as_numpy: bool = True,
                           distributed: Optional[bool] = None):
    """Deep-ensemble predictions (n_models, samples, 1) float32 (inference mode); member-parallel
    over the ranks under ``torchrun`` (``distributed=None`` = auto)."""
    torch = _torch()
    start_time = time.time()
    from . import distributed as D

    if ensemble_models and (D.active() if distributed is None else distributed):
        out = D.deep_ensembles_predict_sharded(ensemble_models, x_test_data)
        out = out.cpu().numpy() if as_numpy else out
    elif ensemble_models and all(getattr(m, "uses_x3", lambda: False)() for m in ensemble_models):
        # fp32-faithful engine, every member in one launch per layer (x3.X3Model with G = M)
        from ..ops import x3

        m0 = ensemble_models[0]
        eng = x3.X3Model(m0.spec, [{k: v.to(m0.device) for k, v in m.store.as_dict().items()}
                                    for m in ensemble_models], device=m0.device)
        out = x3.forward_running(eng, m0._as_input(x_test_data))[:, 0].unsqueeze(-1)
        out = out.cpu().numpy() if as_numpy else out
    elif ensemble_models and all(getattr(m, "uses_fused", lambda: False)() for m in ensemble_models):
        from ..ops import fused

        m0 = ensemble_models[0]
        x = m0._as_input(x_test_data).to(torch.bfloat16).contiguous()
        blobs = torch.cat([m.fused_blob().to(m0.device) for m in ensemble_models])
        out = fused.fused_forward(x, blobs, m0.spec)[:, 0].unsqueeze(-1)
        out = out.float().cpu().numpy() if as_numpy else out
    elif (ensemble_models and all(getattr(m, "uses_tiled_x3", lambda: False)() for m in ensemble_models)
          and all(m.spec == ensemble_models[0].spec for m in ensemble_models)):
        # the pooled / single-channel members at fp32: every member in ONE fused fp16x3 launch
        from ..ops import _ext, fused

        _ext.require()
        m0 = ensemble_models[0]
        blobs = torch.cat([m.fused_blob_x3().to(m0.device) for m in ensemble_models])
        out = fused.tiled_x3_forward(m0._as_input(x_test_data), blobs, m0.spec)[:, 0].unsqueeze(-1)
        out = out.cpu().numpy() if as_numpy else out
    elif ensemble_models and all(getattr(m, "uses_hip", lambda: False)() for m in ensemble_models):
        m0 = ensemble_models[0]
        x = m0._as_input(x_test_data)
        out = torch.stack([m.hip_infer(x.to(m.device))[0].to(m0.device) for m in ensemble_models]).unsqueeze(-1)
        out = out.float().cpu().numpy() if as_numpy else out
    else:
        preds = [np.asarray(m.predict(x_test_data, verbose=0)) for m in ensemble_models]
        out = np.stack(preds) if as_numpy else torch.as_tensor(np.stack(preds))
    print(f"Deep Ensemble completed in {time.time() - start_time:.1f}s ({len(ensemble_models)} models)")
    return out


# ===================== Uncertainty Metrics =====================
def safe_entropy(probs: np.ndarray, axis: int = 1, epsilon: float = 1e-10) -> np.ndarray:
    """Entropy (nats) of probability rows after clipping to [eps, 1-eps] (SciPy renormalises)."""
    return entropy(np.clip(probs, epsilon, 1 - epsilon), axis=axis)


def _device_windows(predictions):
    """Per-window metrics on the GPU: returns (metrics (7, N) cuda tensor, predictions 2-D tensor)."""
    torch = _torch()
    from ..ops import uq as uq_ops

    p = predictions if isinstance(predictions, torch.Tensor) else torch.as_tensor(M.as_2d(predictions))
    if p.dim() == 3 and p.shape[-1] == 1:
        p = p[..., 0]
    if p.dim() == 1:
        p = p.reshape(1, -1)
    p = p.to("cuda", torch.float32).contiguous()
    return uq_ops.metrics(p), p


def uq_evaluation_dist(uq_predictions, y_true) -> Dict[str, np.ndarray]:
    """Per-sample and aggregate UQ metrics (same 8 keys as the reference)."""
    torch = _torch()
    p2 = uq_predictions
    use_dev = isinstance(p2, torch.Tensor) and p2.is_cuda
    if not use_dev and np.asarray(p2).size >= 1_000_000 and _gpu_ok():
        use_dev = True
    y = np.asarray(y_true.cpu() if isinstance(y_true, torch.Tensor) else y_true)
    if use_dev:
        from ..ops import uq as uq_ops

        mt, p = _device_windows(p2)
        if p.shape[0] == 1:
            print("Warning: Only one set of predictions provided. Variance and Mutual Info will be zero.")
        mm = mt.cpu().numpy()
        w = {"mean_pred": mm[uq_ops.MEAN], "pred_variance": mm[uq_ops.VAR], "total_pred_entropy": mm[uq_ops.ENT_NATS],
             "expected_aleatoric_entropy": mm[uq_ops.EXP_ENT], "mutual_info": mm[uq_ops.MI]}
    else:
        p = M.as_2d(np.asarray(p2.cpu() if isinstance(p2, torch.Tensor) else p2))
        if p.shape[0] == 1:
            print("Warning: Only one set of predictions provided. Variance and Mutual Info will be zero.")
        w = M.per_window(p)
    agg = M.aggregates(w, y)
    return {**w, "overall_mean_variance": agg["overall_mean_variance"],
            "mean_variance_class_0": agg["mean_variance_class_0"],
            "mean_variance_class_1": agg["mean_variance_class_1"]}


# ===================== Confidence Intervals =====================
def bootstrap_metrics(uq_predictions, y_true, n_bootstrap: int = 100, random_state: Optional[int] = None,
                      parity: bool = True, device: Optional[str] = None,
                      distributed: bool = False) -> Optional[List[Dict]]:
    """B bootstrap replicates of the 6 aggregate UQ metrics.

    The per-window metrics are invariant under resampling, so each replicate is a gather + mean
    over the resampled windows (mathematically identical to the reference's full recomputation,
    ``uq_techniques.py:137-157``).  ``distributed=True`` shards the windows over the process group and
    all-reduces the replicate sums (``distributed.bootstrap_sharded``); it is a collective, so
    EVERY rank must call it.  Sharding divides the window data and the per-window metric pass; every rank
    still enumerates all B x n draws (cheap integer work) and keeps those landing in its shard.  The default is the local computation: the drivers reach this function on
    rank 0 only (``drivers._finish``), where a collective would wait for the other ranks forever.
    """
    torch = _torch()
    p = uq_predictions
    n_samples = (p.shape[1] if p.ndim >= 2 else p.shape[0])
    y = np.asarray(y_true.cpu() if isinstance(y_true, torch.Tensor) else y_true)
    print(f"Starting bootstrap with {n_bootstrap} iterations...")
    use_dev = (device == "cuda") or (device is None and ((isinstance(p, torch.Tensor) and p.is_cuda) or _gpu_ok()))
    from . import distributed as D

    try:
        if distributed and D.active():
            idx = M.parity_bootstrap_indices(n_samples, n_bootstrap, random_state) if parity else None
            res = D.bootstrap_sharded(p, y, n_bootstrap, seed=0 if random_state is None else random_state, idx=idx)
            out = [dict(zip(M.AGG_KEYS, (float(v) for v in row))) for row in res.cpu().numpy()]
        elif use_dev:
            from ..ops import uq as uq_ops

            mt, _ = _device_windows(p)
            yt = torch.as_tensor(y.astype(np.int32), device="cuda")
            idx = None
            if parity:
                idx = torch.as_tensor(M.parity_bootstrap_indices(n_samples, n_bootstrap, random_state).astype(np.int32),
                                      device="cuda")
            res = uq_ops.bootstrap(mt, yt, n_bootstrap, idx=idx, seed=0 if random_state is None else random_state)
            res = res.cpu().numpy()
            out = [dict(zip(M.AGG_KEYS, (float(v) for v in row))) for row in res]
        else:
            w = M.per_window(np.asarray(p.cpu() if isinstance(p, torch.Tensor) else p))
            if parity:
                idx = M.parity_bootstrap_indices(n_samples, n_bootstrap, random_state)
            else:
                from ..ops import uq as uq_ops

                idx = uq_ops._hash_idx(n_samples, n_bootstrap, 0 if random_state is None else random_state, "cpu").numpy()
            out = M.bootstrap_from_windows(w, y, idx)
    except Exception as e:  # reference tolerates failures per iteration (uq_techniques.py:162-165)
        print(f"Error during bootstrap: {e}")
        return None
    if not out:
        print("Error: No bootstrap results generated.")
        return None
    print("Bootstrap finished.")
    return out


def compute_confidence_intervals(bootstrap_results: List[Dict], alpha: float = 0.05) -> Dict[str, float]:
    """``{m}_mean``, ``{m}_ci_lower``, ``{m}_ci_upper`` percentile intervals per metric."""
    return M.confidence_intervals(bootstrap_results, alpha)


# ===================== Visualization Functions =====================
def plot_uncertainty_metric(uncertainty_values: np.ndarray, uq_name: str, metric_name: str,
                            output_dir: str = "./uq_plots", title: Optional[str] = None, max_samples: int = 5000):
    if plt is None:
        return
    os.makedirs(output_dir, exist_ok=True)
    vals = np.asarray(uncertainty_values)
    n = len(vals)
    idx = np.arange(n)
    if n > max_samples:
        sel = np.sort(np.random.choice(n, max_samples, replace=False))
        vals, idx = vals[sel], idx[sel]
        print(f"Warning: Plotting line plot for {max_samples} random samples out of {n}.")
    fig = plt.figure(figsize=(15, 4))
    plt.plot(idx, vals, alpha=0.7)
    plt.title(title or f"{metric_name} over Samples - {uq_name}")
    plt.xlabel("Sample Index (Subsampled)" if n > max_samples else "Sample Index")
    plt.ylabel(metric_name)
    plt.grid(True, alpha=0.3)
    plt.tight_layout()
    plt.savefig(os.path.join(output_dir, f"line_{metric_name}_{uq_name}.png"), bbox_inches="tight")
    plt.close(fig)


def plot_class_uncertainties(class0_unc: float, class1_unc: float, uq_name: str, output_dir: str = "./uq_plots"):
    if plt is None:
        return
    os.makedirs(output_dir, exist_ok=True)
    fig = plt.figure(figsize=(6, 5))
    bars = plt.bar(["Normal (0)", "Apnea/Hypopnea (1)"], [class0_unc, class1_unc], color=["skyblue", "salmon"])
    plt.bar_label(bars, fmt="%.6f")
    plt.title(f"Mean Predictive Variance by True Class - {uq_name}")
    plt.ylabel("Mean Predictive Variance")
    plt.ylim(bottom=0)
    plt.tight_layout()
    plt.savefig(os.path.join(output_dir, f"bar_class_variance_{uq_name}.png"), bbox_inches="tight")
    plt.close(fig)


def plot_metric_distribution(metric_values: np.ndarray, y_true: np.ndarray, uq_name: str, metric_name: str,
                             output_dir: str = "./uq_plots", bins: int = 30):
    if plt is None:
        return
    os.makedirs(output_dir, exist_ok=True)
    v, y = np.asarray(metric_values), np.asarray(y_true)
    fig = plt.figure(figsize=(10, 6))
    if np.any(y == 0):
        plt.hist(v[y == 0], bins=bins, alpha=0.6, label="True Normal (0)", density=True)
    if np.any(y == 1):
        plt.hist(v[y == 1], bins=bins, alpha=0.6, label="True Apnea/Hypopnea (1)", density=True)
    plt.title(f"{metric_name} Distribution by True Class - {uq_name}")
    plt.xlabel(f"{metric_name} Value")
    plt.ylabel("Density")
    plt.legend()
    plt.grid(True, alpha=0.3)
    plt.tight_layout()
    plt.savefig(os.path.join(output_dir, f"hist_{metric_name}_by_class_{uq_name}.png"), bbox_inches="tight")
    plt.close(fig)


# ===================== Main Evaluation Function =====================
def evaluate_uq_methods(predictions, y_test, evaluation_label: str = "UQ Evaluation", n_bootstrap: int = 100,
                        random_state: Optional[int] = None, output_plot_dir: str = "./uq_plots",
                        make_plots: bool = True, parity: bool = True) -> Optional[Dict]:
    """Metrics + bootstrap CIs + plots; returns the reference's 24-key dictionary."""
    torch = _torch()
    print(f"\n=== Evaluating Uncertainty: {evaluation_label} ===")
    if predictions is None or y_test is None:
        print("Error: Input predictions or labels are None.")
        return None
    print(f"Input prediction shape: {tuple(predictions.shape)}, Samples: {len(y_test)}")
    if len(y_test) != predictions.shape[1]:
        raise ValueError(f"Mismatch between prediction samples ({predictions.shape[1]}) and label samples ({len(y_test)})")
    if predictions.ndim == 3 and predictions.shape[-1] == 1:
        predictions = predictions[..., 0]
    if predictions.ndim == 1:
        predictions = predictions.reshape(1, -1)
    print("\nCalculating base UQ metrics...")
    w = uq_evaluation_dist(predictions, y_test)
    pt = {
        "overall_mean_variance": w["overall_mean_variance"],
        "mean_variance_class_0": w["mean_variance_class_0"],
        "mean_variance_class_1": w["mean_variance_class_1"],
        "mean_total_pred_entropy": float(np.mean(w["total_pred_entropy"])),
        "mean_expected_aleatoric_entropy": float(np.mean(w["expected_aleatoric_entropy"])),
        "mean_mutual_info": float(np.mean(w["mutual_info"])),
    }
    print(f"- Overall Mean Variance: {pt['overall_mean_variance']:.6f}")
    print(f"- Mean Variance Class 0: {pt['mean_variance_class_0']:.6f}")
    print(f"- Mean Variance Class 1: {pt['mean_variance_class_1']:.6f}")
    print(f"- Mean Predictive Entropy (Total): {pt['mean_total_pred_entropy']:.4f}")
    print(f"- Mean Expected Entropy (Aleatoric): {pt['mean_expected_aleatoric_entropy']:.4f}")
    print(f"- Mean Mutual Info (Epistemic): {pt['mean_mutual_info']:.6f}")
    print(f"\nComputing CIs (n_bootstrap={n_bootstrap})...")
    t0 = time.time()
    boot = bootstrap_metrics(predictions, y_test, n_bootstrap, random_state, parity=parity)
    final: Dict[str, float] = {}
    if boot:
        final.update(compute_confidence_intervals(boot))
        print(f"CIs computed in {time.time() - t0:.2f}s")
    else:
        print("Warning: Bootstrap failed, CIs not computed.")
    final.update(pt)
    if make_plots:
        print("\nGenerating visualizations...")
        y = np.asarray(y_test.cpu() if isinstance(y_test, torch.Tensor) else y_test)
        plot_metric_distribution(w["pred_variance"], y, evaluation_label, "Predictive Variance", output_dir=output_plot_dir)
        plot_metric_distribution(w["total_pred_entropy"], y, evaluation_label, "Predictive Entropy",
                                 output_dir=output_plot_dir)
        plot_metric_distribution(w["mutual_info"], y, evaluation_label, "Mutual Information", output_dir=output_plot_dir)
        plot_class_uncertainties(final["mean_variance_class_0"], final["mean_variance_class_1"], evaluation_label,
                                 output_dir=output_plot_dir)
    print("\n=== Evaluation Complete ===")
    return final


def demo(output_plot_dir: str = "./dummy_uq_plots", n_models: int = 5, n_samples: int = 1000, seed: int = 42):
    """The reference's synthetic smoke run (``uq_techniques.py:395-446``), same data recipe."""
    rs = np.random.RandomState(seed)
    preds = []
    for _ in range(n_models):
        p = rs.rand(n_samples) * 0.6 + 0.2
        noise = rs.randn(n_samples) * 0.1
        preds.append(np.clip(p + noise, 0.01, 0.99))
    preds = np.stack(preds)
    labels = (rs.rand(n_samples) > 0.7).astype(int)
    return evaluate_uq_methods(preds, labels, "Dummy Ensemble Test", n_bootstrap=50, random_state=seed,
                               output_plot_dir=output_plot_dir)


if __name__ == "__main__":
    res = demo()
    for k, v in (res or {}).items():
        print(f"{k}: {v:.6f}")
