"""Patient- and window-level post-hoc analyses of the per-window UQ CSV.

* :func:`aggregate_patient_uq_metrics` — ``aggregate_patient_uq_metrics.py:16-83``: per patient
  mean / median / std of variance and entropy, accuracy and window count (std := 0 for a
  single-window patient); summary CSV + textual report (top/bottom patients by mean entropy).
* :func:`window_level_binning` — ``analyze_window_level_uncertainty.py:40-67``: correct vs incorrect
  descriptive statistics and 10 equal-width entropy bins ``linspace(min, max + 1e-9)`` with
  ``pd.cut(right=False)``; accuracy and error rate per bin.
"""
from __future__ import annotations

import os
from typing import Optional, Union

import numpy as np
import pandas as pd

REQUIRED = ["Patient_ID", "True_Label", "Predicted_Label", "Predictive_Variance", "Predictive_Entropy"]


def _load(df_or_csv: Union[str, pd.DataFrame]) -> pd.DataFrame:
    return pd.read_csv(df_or_csv) if isinstance(df_or_csv, str) else df_or_csv.copy()


def aggregate_patient_uq_metrics(detail: Union[str, pd.DataFrame], output_dir: Optional[str] = None,
                                 tag: str = "MCD", n_examples: int = 5, verbose: bool = True) -> pd.DataFrame:
    df = _load(detail)
    missing = [c for c in REQUIRED if c not in df.columns]
    if missing:
        raise ValueError(f"Missing one or more required columns: {missing}")
    df["Correct"] = df["True_Label"] == df["Predicted_Label"]
    s = df.groupby("Patient_ID").agg(
        mean_variance=("Predictive_Variance", "mean"),
        median_variance=("Predictive_Variance", "median"),
        std_variance=("Predictive_Variance", "std"),
        mean_entropy=("Predictive_Entropy", "mean"),
        median_entropy=("Predictive_Entropy", "median"),
        std_entropy=("Predictive_Entropy", "std"),
        patient_accuracy=("Correct", "mean"),
        num_windows=("Patient_ID", "size"),
    ).reset_index()
    single = s["num_windows"] <= 1
    s.loc[single, "std_variance"] = 0.0
    s.loc[single, "std_entropy"] = 0.0
    if output_dir:
        os.makedirs(output_dir, exist_ok=True)
        path = os.path.join(output_dir, f"patient_summary_metrics_{tag}.csv")
        s.to_csv(path, index=False)
        if verbose:
            print(f"\nSaved patient summary metrics to: {path}")
    if verbose:
        cols = ["mean_entropy", "mean_variance", "std_entropy", "std_variance", "patient_accuracy"]
        print(f"\nNumber of unique patients in summary: {len(s)}")
        print("\nOverall Patient Statistics:")
        print(s[cols].describe().to_string())
        srt = s.sort_values("mean_entropy", ascending=False)
        show = ["Patient_ID", "mean_entropy", "mean_variance", "patient_accuracy", "num_windows"]
        print(f"\nTop {n_examples} Patients with HIGHEST Mean Entropy:")
        print(srt.head(n_examples)[show].to_string())
        print(f"\nTop {n_examples} Patients with LOWEST Mean Entropy:")
        print(srt.tail(n_examples)[show].to_string())
        print("\nStatistics for HIGHEST Mean Entropy Group:")
        print(srt.head(n_examples)[cols].describe().to_string())
        print("\nStatistics for LOWEST Mean Entropy Group:")
        print(srt.tail(n_examples)[cols].describe().to_string())
    return s


def window_level_binning(detail: Union[str, pd.DataFrame], metric: str = "Predictive_Entropy", num_bins: int = 10,
                         verbose: bool = True) -> pd.DataFrame:
    df = _load(detail)
    if "Correct" not in df.columns:
        df["Correct"] = df["True_Label"] == df["Predicted_Label"]
    if verbose:
        print(f"\nTotal number of windows analyzed: {len(df)}")
        print(f"Overall accuracy across all windows: {df['Correct'].mean():.4f}")
        print("\nStatistics for CORRECTLY Classified Windows:")
        print(df[df["Correct"]][["Predictive_Entropy", "Predictive_Variance"]].describe().to_string())
        print("\nStatistics for INCORRECTLY Classified Windows:")
        print(df[~df["Correct"]][["Predictive_Entropy", "Predictive_Variance"]].describe().to_string())
    lo, hi = df[metric].min(), df[metric].max()
    bins = np.linspace(lo, hi + 1e-9, num_bins + 1)
    labels = [f"{bins[i]:.3f}-{bins[i + 1]:.3f}" for i in range(num_bins)]
    df[f"{metric}_Bin"] = pd.cut(df[metric], bins=bins, labels=labels, right=False)
    out = df.groupby(f"{metric}_Bin", observed=False).agg(window_count=("Correct", "size"),
                                                          accuracy=("Correct", "mean"))
    out["error_rate"] = 1 - out["accuracy"]
    if verbose:
        print(f"\nAccuracy and Error Rate per {metric} Bin:")
        print(out.to_string(float_format="%.4f"))
    return out
