"""Thesis figures (``uq_analysis/final_plot_uq_overview_figures.py``, ``hyperparameter_plot_...``).

seaborn is not available; the same four figures are drawn with matplotlib (+ a SciPy Gaussian KDE
for the histogram overlay):

1. ``patient_entropy_histograms_final.png`` — per-patient mean entropy, MCD vs DE (20 bins + KDE);
2. ``patient_accuracy_vs_entropy_final.png`` — patient accuracy vs mean entropy with Pearson r
   (NaNs dropped jointly, fixing SURVEY Q12);
3. ``window_correctness_boxplots_final.png`` — entropy of correct vs incorrect windows;
4. ``binned_accuracy_plot_final_annotated.png`` — accuracy over 10 entropy bins, first bin starred.

plus :func:`plot_variance_convergence` (overall mean variance vs passes / members).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import pandas as pd

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
from scipy.stats import gaussian_kde, pearsonr  # noqa: E402


def load_data(csv_path: str) -> Optional[pd.DataFrame]:
    """``final_plot_uq_overview_figures.py:26-37``: the CSV as a DataFrame, or None if it is missing
    or unreadable (reported, not raised)."""
    if not os.path.exists(csv_path):
        print(f"ERROR: File not found - {csv_path}")
        return None
    try:
        df = pd.read_csv(csv_path)
    except Exception as e:  # noqa: BLE001 -- the reference reports and returns None
        print(f"Error loading {csv_path}: {e}")
        return None
    print(f"Loaded {csv_path}, shape: {df.shape}")
    return df


def _hist_kde(ax, v, bins=20):
    v = np.asarray(v, dtype=float)
    v = v[np.isfinite(v)]
    cnt, edges, _ = ax.hist(v, bins=bins, alpha=0.6, edgecolor="white")
    if v.size > 1 and np.std(v) > 0:
        xs = np.linspace(v.min(), v.max(), 200)
        ax.plot(xs, gaussian_kde(v)(xs) * v.size * (edges[1] - edges[0]))


def _correct(df):
    if "Correct" not in df.columns:
        df["Correct"] = df["True_Label"] == df["Predicted_Label"]
    return df


def final_overview_figures(mcd_detail: Optional[pd.DataFrame], de_detail: Optional[pd.DataFrame],
                           mcd_summary: Optional[pd.DataFrame], de_summary: Optional[pd.DataFrame],
                           out_dir: str = "./final_thesis_plots", dpi: int = 150):
    os.makedirs(out_dir, exist_ok=True)
    written = []
    if mcd_summary is not None and de_summary is not None:
        fig, ax = plt.subplots(1, 2, figsize=(12, 5), sharey=True)
        for a, df, t in zip(ax, [mcd_summary, de_summary], ["a) MC Dropout", "b) Deep Ensemble"]):
            _hist_kde(a, df["mean_entropy"])
            a.set_title(t)
            a.set_xlabel("Mean Predictive Entropy per Patient")
        ax[0].set_ylabel("Number of Patients")
        fig.suptitle("Distribution of Mean Predictive Entropy Across Patients (Unbalanced Set)")
        fig.tight_layout(rect=[0, 0.03, 1, 0.95])
        p = os.path.join(out_dir, "patient_entropy_histograms_final.png")
        fig.savefig(p, dpi=dpi)
        plt.close(fig)
        written.append(p)

        fig, ax = plt.subplots(1, 2, figsize=(12, 5.5))
        for a, df, t in zip(ax, [mcd_summary, de_summary], ["a) MC Dropout", "b) Deep Ensemble"]):
            c = df[["mean_entropy", "patient_accuracy"]].dropna()
            r = pearsonr(c["mean_entropy"], c["patient_accuracy"])[0] if len(c) > 1 else float("nan")
            a.scatter(c["mean_entropy"], c["patient_accuracy"], alpha=0.6, s=14)
            a.set_title(t)
            a.set_xlabel("Mean Predictive Entropy per Patient")
            a.set_ylabel("Patient Accuracy")
            a.text(0.95, 0.05, f"Pearson r = {r:.3f}", transform=a.transAxes, fontsize=9, ha="right", va="bottom")
            a.grid(True, linestyle="--", alpha=0.6)
        fig.suptitle("Patient Accuracy vs. Mean Predictive Entropy (Unbalanced Set)")
        fig.tight_layout(rect=[0, 0.03, 1, 0.95])
        p = os.path.join(out_dir, "patient_accuracy_vs_entropy_final.png")
        fig.savefig(p, dpi=dpi)
        plt.close(fig)
        written.append(p)
    if mcd_detail is not None and de_detail is not None:
        mcd_detail, de_detail = _correct(mcd_detail.copy()), _correct(de_detail.copy())
        fig, ax = plt.subplots(1, 2, figsize=(10, 5))
        for a, df, t in zip(ax, [mcd_detail, de_detail], ["a) MC Dropout", "b) Deep Ensemble"]):
            a.boxplot([df.loc[df["Correct"], "Predictive_Entropy"].dropna(),
                       df.loc[~df["Correct"], "Predictive_Entropy"].dropna()], tick_labels=["Correct", "Incorrect"])
            a.set_title(t)
            a.set_xlabel("Prediction Correct")
            a.set_ylabel("Predictive Entropy")
        fig.suptitle("Predictive Entropy Distribution for Correct vs. Incorrect Windows (Unbalanced Set)")
        fig.tight_layout(rect=[0, 0.03, 1, 0.95])
        p = os.path.join(out_dir, "window_correctness_boxplots_final.png")
        fig.savefig(p, dpi=dpi)
        plt.close(fig)
        written.append(p)

        fig, ax = plt.subplots(1, 2, figsize=(14, 6), sharey=True)
        for i, (a, df, name) in enumerate(zip(ax, [mcd_detail, de_detail], ["MC Dropout", "Deep Ensemble"])):
            m = "Predictive_Entropy"
            bins = np.linspace(df[m].min(), df[m].max(), 11)
            bins[-1] += 1e-9
            cut = pd.cut(df[m], bins=bins, include_lowest=True)
            br = df.groupby(cut, observed=False).agg(window_count=("Correct", "size"), accuracy=("Correct", "mean"))
            xs = np.arange(len(br))
            line = a.plot(xs, br["accuracy"], marker="o", linewidth=2)[0]
            a.set_xticks(xs)
            a.set_xticklabels([f"{iv.left:.2f}-{iv.right:.2f}" for iv in br.index], rotation=45, ha="right", fontsize=9)
            acc0, n0 = br["accuracy"].iloc[0], br["window_count"].iloc[0]
            a.plot(0, acc0, marker="*", markersize=12, color=line.get_color(), markeredgecolor="black", zorder=5)
            a.text(0.05, acc0 - 0.08, f"Acc: {acc0:.3f}\nN: {n0:,}", ha="left", va="top", fontsize=9,
                   bbox=dict(boxstyle="round,pad=0.3", fc="white", ec="gray", alpha=0.8))
            a.set_title(f"{'a)' if i == 0 else 'b)'} {name}\n(Overall UQ run Acc: {df['Correct'].mean():.2f})", fontsize=11)
            a.set_xlabel("Predictive Entropy Bin")
            if i == 0:
                a.set_ylabel("Accuracy")
            a.grid(True, linestyle="--", alpha=0.7)
            a.set_ylim(0.5, 1.05)
        fig.suptitle("Accuracy across Predictive Entropy Bins (Unbalanced Set)", fontsize=14)
        fig.tight_layout(rect=[0, 0.03, 1, 0.93])
        p = os.path.join(out_dir, "binned_accuracy_plot_final_annotated.png")
        fig.savefig(p, dpi=dpi)
        plt.close(fig)
        written.append(p)
    return written


def plot_variance_convergence(convergence_data_csv: str, output_plot_filename: str = "variance_convergence_plot.png",
                              method: str = "mcd", dpi: int = 300) -> Optional[str]:
    df = pd.read_csv(convergence_data_csv)
    req = ["N", "Variance_Unbalanced", "Variance_Balanced"]
    if any(c not in df.columns for c in req) or df.empty:
        print(f"ERROR: Input CSV must have columns {req} and rows")
        return None
    if method.lower() == "mcd":
        title, xl = "MC Dropout: Overall Mean Variance Convergence", "Number of Forward Passes (N)"
    elif method.lower() == "de":
        title, xl = "Deep Ensemble: Overall Mean Variance Convergence", "Number of Ensemble Members"
    else:
        title, xl = "Overall Mean Variance Convergence", "N"
    fig, ax = plt.subplots(figsize=(8, 5))
    ax.plot(df["N"], df["Variance_Unbalanced"], marker="^", linestyle="-", color="forestgreen", label="Variance (Unbalanced)")
    ax.plot(df["N"], df["Variance_Balanced"], marker="v", linestyle="--", color="firebrick", label="Variance (Balanced)")
    ax.set_title(title, fontsize=13, pad=15)
    ax.set_xlabel(xl, fontsize=11)
    ax.set_ylabel("Overall Mean Predictive Variance", fontsize=11)
    ax.legend(fontsize=9)
    ax.grid(True, which="both", linestyle="--", linewidth=0.5)
    ax.set_xticks(df["N"])
    ax.set_ylim(bottom=0)
    fig.tight_layout()
    d = os.path.dirname(output_plot_filename)
    if d:
        os.makedirs(d, exist_ok=True)
    fig.savefig(output_plot_filename, dpi=dpi, bbox_inches="tight")
    plt.close(fig)
    return output_plot_filename
