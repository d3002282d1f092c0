"""Statistical tests of the thesis analysis (``uq_analysis/``).

* :func:`patient_correlation` — ``patient_accuracy_entropy_correlation.py:15-46``: Pearson r between
  a patient summary's ``mean_entropy`` and ``patient_accuracy`` (rows with NaN dropped jointly);
  :func:`calculate_and_print_correlation` is the reference's file-path entry point.
* :func:`entropy_mannwhitney` — ``window_uncertainty_vs_correctness_mannwhitney.py:18``: one-sided
  Mann-Whitney U (incorrect > correct) on per-window predictive entropy.  The reference script is
  labelled "Deep Ensembles" whatever file it reads; here the method is a parameter.
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import pandas as pd
from scipy.stats import mannwhitneyu, pearsonr


def patient_correlation(summary: Union[str, pd.DataFrame], method: str = "MC Dropout", x_col: str = "mean_entropy",
                        y_col: str = "patient_accuracy", verbose: bool = True) -> Tuple[Optional[float], Optional[float]]:
    df = pd.read_csv(summary) if isinstance(summary, str) else summary
    if x_col not in df.columns or y_col not in df.columns:
        print(f"ERROR: Required columns ('{x_col}', '{y_col}') not found")
        return None, None
    clean = df[[x_col, y_col]].dropna()
    if len(clean) < 2:
        print("ERROR: Not enough valid data points for correlation.")
        return None, None
    r, p = pearsonr(clean[x_col], clean[y_col])
    if verbose:
        print(f"--- Analyzing {method} ---")
        print(f"Correlation between '{x_col}' and '{y_col}':")
        print(f"Pearson r = {r:.4f}")
        print(f"P-value = {p:.4g}")
    return float(r), float(p)


def calculate_and_print_correlation(csv_path: str, method_name: str, x_col: str = "mean_entropy",
                                    y_col: str = "patient_accuracy") -> Tuple[Optional[float], Optional[float]]:
    """Reference entry point (``patient_accuracy_entropy_correlation.py:15-46``): (r, p) or (None, None)
    when the file or columns are missing or fewer than two rows survive the joint NaN drop."""
    import os

    if not os.path.exists(csv_path):
        print(f"ERROR: File not found - {csv_path}")
        return None, None
    try:
        df = pd.read_csv(csv_path)
    except Exception as e:  # noqa: BLE001 -- the reference reports and returns (None, None)
        print(f"Error processing {csv_path}: {e}")
        return None, None
    if x_col in df.columns and y_col in df.columns:
        n_drop = len(df) - len(df[[x_col, y_col]].dropna())
        if n_drop:
            print(f"Warning: Dropped {n_drop} rows with NaN values.")
    return patient_correlation(df, method_name, x_col, y_col)


def entropy_mannwhitney(detail: Union[str, pd.DataFrame], method: str = "Deep Ensembles", metric: str = "Predictive_Entropy",
                        verbose: bool = True) -> Tuple[Optional[float], Optional[float]]:
    df = pd.read_csv(detail) if isinstance(detail, str) else detail.copy()
    if "Correct" not in df.columns:
        df["Correct"] = df["True_Label"] == df["Predicted_Label"]
    good = df.loc[df["Correct"] == True, metric].dropna()  # noqa: E712
    bad = df.loc[df["Correct"] == False, metric].dropna()  # noqa: E712
    if len(good) == 0 or len(bad) == 0:
        print("Not enough data in one or both groups to perform the test.")
        return None, None
    stat, p = mannwhitneyu(bad, good, alternative="greater")
    if verbose:
        print(f"\n--- Mann-Whitney U Test Results ({metric}: Incorrect > Correct) ---")
        print(f"Method: {method}")
        print(f"U Statistic: {stat}")
        print(f"P-value: {p: .4g}")
        print("Conclusion: " + ("The difference is statistically significant (p < 0.05)." if p < 0.05
                                else "The difference is not statistically significant (p >= 0.05)."))
    return float(stat), float(p)
