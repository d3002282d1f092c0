"""UQ experiment drivers: per-window results, raw prediction dumps, aggregate metrics + CIs.

Library form of the reference's module-level scripts
(``uncertainty_quantification/analyze_mcd_patient_level.py:71-193``,
``analyze_de_patient_level.py:88-193``, ``evaluate_mcd_global.py``, ``evaluate_de_global.py``):

1. stochastic predictions — MC Dropout T passes (one fused launch, or the reference's batch-BN
   semantics) or the M ensemble members (one fused launch for all members);
2. ``np.save`` of the raw (T|M, N, 1) predictions;
3. per-window mean / variance / entropy in BITS (log2(p + 1e-9)) / label (> 0.5) computed on the
   device by ``uq_reduce``; accuracy of the mean prediction printed;
4. the per-window CSV ``Patient_ID, Window_Index, True_Label, Predicted_Label,
   Predicted_Probability, Predictive_Variance, Predictive_Entropy``;
5. ``evaluate_uq_methods`` (aggregates, bootstrap CIs, plots).

The reference's ``evaluate_mcd_global.py`` runs 3 x T passes where 2 x T suffice (Q11); here each
evaluation reuses its own samples.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import pandas as pd

from . import uq_techniques as U

DETAIL_COLUMNS = ["Patient_ID", "Window_Index", "True_Label", "Predicted_Label", "Predicted_Probability",
                  "Predictive_Variance", "Predictive_Entropy"]


def per_window_table(probs, y, patient_ids=None) -> pd.DataFrame:
    """Per-window DataFrame from (T|M, N[, 1]) probabilities (device reduction when available)."""
    import torch

    from ..ops import uq as uq_ops

    p = probs if isinstance(probs, torch.Tensor) else torch.as_tensor(np.asarray(probs))
    if p.dim() == 3:
        p = p[..., 0]
    if torch.cuda.is_available():
        p = p.cuda()
    m = uq_ops.metrics(p.float()).cpu().numpy()
    y = np.asarray(y)
    mean = m[uq_ops.MEAN]
    return pd.DataFrame({
        "Patient_ID": patient_ids if patient_ids is not None else np.nan,
        "Window_Index": np.arange(len(y)),
        "True_Label": y,
        "Predicted_Label": (mean > 0.5).astype(int),
        "Predicted_Probability": mean,
        "Predictive_Variance": m[uq_ops.VAR],
        "Predictive_Entropy": m[uq_ops.ENT_BITS],
    })


def _main_rank() -> bool:
    from . import distributed as D

    if not D.active():
        return True
    import torch.distributed as dist

    return dist.get_rank() == 0


def _finish(probs_np, y, patient_ids, label, save_detailed_csv, output_csv_dir, output_plot_dir, n_bootstrap, seed,
            raw_pred_path, make_plots) -> Optional[Dict]:
    if not _main_rank():
        return None  # under torchrun every rank holds the gathered samples; rank 0 writes the outputs
    if raw_pred_path:
        d = os.path.dirname(raw_pred_path)
        if d:
            os.makedirs(d, exist_ok=True)
        np.save(raw_pred_path, probs_np)
        print(f"Saved raw predictions (shape: {probs_np.shape}) to {raw_pred_path}")
    df = per_window_table(probs_np, y, patient_ids)
    acc = float((df["Predicted_Label"].values == np.asarray(y)).mean())
    print(f"Accuracy based on mean probability (>0.5): {acc:.4f}")
    if save_detailed_csv:
        if patient_ids is None:
            print("Skipping detailed CSV save because patient IDs were not provided.")
        else:
            os.makedirs(output_csv_dir, exist_ok=True)
            path = os.path.join(output_csv_dir, f"detailed_results_{label}.csv")
            df.to_csv(path, index=False)
            print(f"Saving detailed results to: {path}")
    metrics = U.evaluate_uq_methods(probs_np, y, label, n_bootstrap=n_bootstrap, random_state=seed,
                                    output_plot_dir=os.path.join(output_plot_dir, label), make_plots=make_plots)
    if metrics is not None:
        metrics["accuracy_mean_prediction"] = acc
    return metrics


def evaluate_mc_dropout(model, X, y, patient_ids=None, model_eval_label: str = "CNN_MCD", save_detailed_csv: bool = False,
                        n_passes: int = 50, n_bootstrap: int = 100, seed: int = 2025, bn_mode: str = "batch",
                        output_csv_dir: str = "./uq_results_patient_no_pool",
                        output_plot_dir: str = "./uq_plots_patient/mc_dropout_no_pool",
                        raw_pred_path: Optional[str] = None, make_plots: bool = True) -> Optional[Dict]:
    print(f"\n===== Running MC Dropout Evaluation for: {model_eval_label} =====")
    probs = U.mc_dropout_predict(model, X, n_pred=n_passes, bn_mode=bn_mode, seed=seed)
    if probs is None or probs.shape[0] != n_passes or probs.shape[1] != len(y):
        print(f"MC Dropout prediction failed or returned unexpected shape for {model_eval_label}")
        return None
    if raw_pred_path is None:  # "" skips the dump
        raw_pred_path = f"./mc_raw_pred0505_{model_eval_label}.npy"
    return _finish(probs, y, patient_ids, model_eval_label, save_detailed_csv, output_csv_dir, output_plot_dir,
                   n_bootstrap, seed, raw_pred_path, make_plots)


def evaluate_deep_ensemble(models: List, X, y, patient_ids=None, model_eval_label: str = "CNN_DE",
                           save_detailed_csv: bool = False, n_bootstrap: int = 100, seed: int = 2025,
                           output_csv_dir: str = "./uq_results_patient_DE_new",
                           output_plot_dir: str = "./uq_plots_patient/deep_ensemble_no_pool",
                           raw_pred_path: Optional[str] = "", make_plots: bool = True) -> Optional[Dict]:
    print(f"\n===== Running Deep Ensemble Evaluation for: {model_eval_label} =====")
    if not models:
        print("ERROR: No models provided in the ensemble list.")
        return None
    probs = U.deep_ensembles_predict(models, X)
    if probs is None or probs.shape[0] != len(models) or probs.shape[1] != len(y):
        print(f"Deep Ensemble prediction failed or returned unexpected shape for {model_eval_label}")
        return None
    return _finish(probs, y, patient_ids, model_eval_label, save_detailed_csv, output_csv_dir, output_plot_dir,
                   n_bootstrap, seed, raw_pred_path, make_plots)


def evaluate_mc_dropout_global(model, X_data_reshaped, y_data, model_eval_label: str, n_passes: int = 50,
                               n_bootstrap: int = 100, seed: int = 2025, bn_mode: str = "batch",
                               output_plot_dir: str = "./uq_plots/mc_dropout", make_plots: bool = True) -> Optional[Dict]:
    """``evaluate_mcd_global.py:45-94`` signature ``evaluate_mc_dropout(model, X, y, label)``: MC Dropout
    + ``evaluate_uq_methods``, no per-window CSV or raw dump (exported under the reference name by
    ``cli/evaluate_mcd_global.py``)."""
    return evaluate_mc_dropout(model, X_data_reshaped, y_data, None, model_eval_label, save_detailed_csv=False,
                               n_passes=n_passes, n_bootstrap=n_bootstrap, seed=seed, bn_mode=bn_mode,
                               output_plot_dir=output_plot_dir, raw_pred_path="", make_plots=make_plots)


def evaluate_ensemble(models: List, X_data, y_data, model_eval_label: str, n_bootstrap: int = 100, seed: int = 2025,
                      output_plot_dir: str = "./uq_plots/deep_ensemble", make_plots: bool = True) -> Optional[Dict]:
    """``evaluate_de_global.py:40-80``: Deep Ensemble predictions + ``evaluate_uq_methods`` for a 3-D
    window array (anything else is rejected, ``:48-50``)."""
    if np.ndim(X_data) != 3:
        print(f"ERROR: Expected 3D input data (samples, steps, features) for model, but got shape {np.shape(X_data)}")
        return None
    return evaluate_deep_ensemble(models, X_data, y_data, None, model_eval_label, save_detailed_csv=False,
                                  n_bootstrap=n_bootstrap, seed=seed, output_plot_dir=output_plot_dir,
                                  raw_pred_path="", make_plots=make_plots)


def convergence_sweep(predict_fn, counts, X_unbalanced, y_unbalanced, X_balanced, y_balanced, output_csv: str):
    """Overall mean variance vs number of passes / members -> ``N, Variance_Unbalanced, Variance_Balanced``.

    The reference's convergence CSV was produced by hand; this computes it.
    ``predict_fn(X, n) -> (n, N[, 1])`` probabilities.
    """
    from . import metrics as M

    rows = []
    for n in counts:
        vu = float(np.mean(M.per_window(predict_fn(X_unbalanced, n))["pred_variance"]))
        vb = float(np.mean(M.per_window(predict_fn(X_balanced, n))["pred_variance"]))
        rows.append({"N": n, "Variance_Unbalanced": vu, "Variance_Balanced": vb})
    df = pd.DataFrame(rows)
    d = os.path.dirname(output_csv)
    if d:
        os.makedirs(d, exist_ok=True)
    df.to_csv(output_csv, index=False)
    return df
