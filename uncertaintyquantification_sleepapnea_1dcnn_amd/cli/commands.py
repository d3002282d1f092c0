"""Command-line entry points mirroring every reference script (same flag names and defaults).

``python -m uncertaintyquantification_sleepapnea_1dcnn_amd <command> [flags]`` or
``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.<command> [flags]``.

| command | reference script |
|---|---|
| preprocess_shhs_raw | data_prepocessing/preprocess_shhs_raw.py |
| prepare_numpy_datasets | data_prepocessing/prepare_numpy_datasets.py |
| cnn_baseline_train | models/cnn_baseline_train.py |
| train_deep_ensemble_cnns | models/train_deep_ensemble_cnns.py (torchrun: one member per GPU) |
| analyze_mcd_patient_level | uncertainty_quantification/analyze_mcd_patient_level.py |
| analyze_de_patient_level | uncertainty_quantification/analyze_de_patient_level.py |
| evaluate_mcd_global | uncertainty_quantification/evaluate_mcd_global.py |
| evaluate_de_global | uncertainty_quantification/evaluate_de_global.py |
| aggregate_patient_uq_metrics | uncertainty_quantification/aggregate_patient_uq_metrics.py |
| analyze_window_level_uncertainty | uncertainty_quantification/analyze_window_level_uncertainty.py |
| final_plot_uq_overview_figures | uq_analysis/final_plot_uq_overview_figures.py |
| patient_accuracy_entropy_correlation | uq_analysis/patient_accuracy_entropy_correlation.py |
| window_uncertainty_vs_correctness_mannwhitney | uq_analysis/window_uncertainty_vs_correctness_mannwhitney.py |
| hyperparameter_plot_mcd_or_de_pass_convergence | uq_analysis/hyperparameter_plot_mcd_or_de_pass_convergence.py |
| convergence_sweep | (new) computes the convergence CSV the reference produced by hand |
| shhs_cohort_analysis / shhs_signal_quality | datasets/SHHS_cohort_analysis.py / SHHS_signal_quality.py |
| uq_demo | uq_techniques.py ``__main__`` demo |
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

SEED = 2025


def preprocess_shhs_raw(argv=None):
    from ..data.preprocess import main

    main(argv)


def prepare_numpy_datasets(argv=None):
    from ..data.prepare import main

    main(argv)


def cnn_baseline_train(argv=None):
    from ..training.experiment import main

    main(argv)


def train_deep_ensemble_cnns(argv=None):
    ap = argparse.ArgumentParser(description="Train CNN ensemble models (member-parallel over GPUs under torchrun).")
    ap.add_argument("--model_type", type=str, default="cnn", help="Type of model to train (only 'cnn' supported).")
    ap.add_argument("--num_models", type=int, default=5)
    ap.add_argument("--seed_base", type=int, default=SEED)
    ap.add_argument("--data_dir", type=str, default="./processed_datasets")
    ap.add_argument("--save_dir", type=str, default="./models/ensemble_cnn_no_pool")
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--batch_size", type=int, default=1024)
    ap.add_argument("--patience", type=int, default=5)
    ap.add_argument("--name_offset", type=int, default=21)
    a = ap.parse_args(argv)
    if a.model_type.lower() != "cnn":
        print(f"Error: This script is configured to train only 'cnn' models, but received '{a.model_type}'.")
        return
    from ..data.prepare import load_processed
    from ..parallel.ensemble import train_ensemble

    X = load_processed(a.data_dir, "X_train_win_std_smote.npy")
    y = load_processed(a.data_dir, "y_train_smote.npy").astype(np.float32)
    train_ensemble(X, y, a.num_models, a.seed_base, a.save_dir, name_offset=a.name_offset, epochs=a.epochs,
                   batch_size=a.batch_size, patience=a.patience)


def reference_train_ensemble(model_type: str = "cnn", num_models: int = 5, seed_base: int = SEED,
                             data_dir: str = "./processed_datasets", save_dir: str = "./models/ensemble_cnn_no_pool"):
    """``train_deep_ensemble_cnns.py:81`` signature ``train_ensemble(model_type, num_models, seed_base)``:
    loads the SMOTE training set from ``data_dir`` and trains the members (skip-if-exists resume)."""
    argv = ["--model_type", model_type, "--num_models", str(num_models), "--seed_base", str(seed_base),
            "--data_dir", data_dir, "--save_dir", save_dir]
    train_deep_ensemble_cnns(argv)


def _load_test(data_dir):
    from ..data.prepare import load_processed

    Xu = load_processed(data_dir, "X_test_win_std_unbalanced.npy")
    yu = load_processed(data_dir, "y_test_unbalanced.npy")
    try:
        pids = load_processed(data_dir, "patient_ids_test_unbalanced.npy")
    except FileNotFoundError:
        pids = None
    Xr = load_processed(data_dir, "X_test_win_std_rus.npy")
    yr = load_processed(data_dir, "y_test_rus.npy")
    return Xu, yu, pids, Xr, yr


def _uq_common(ap):
    ap.add_argument("--data_dir", type=str, default="./processed_datasets")
    ap.add_argument("--n_bootstrap", type=int, default=100)
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--no_plots", action="store_true")


def analyze_mcd_patient_level(argv=None, global_mode: bool = False):
    ap = argparse.ArgumentParser(description="MC Dropout UQ evaluation with per-window results.")
    _uq_common(ap)
    ap.add_argument("--model_path", type=str, default="./AlCNN1D_no_pool.keras")
    ap.add_argument("--n_passes", type=int, default=50)
    ap.add_argument("--bn_mode", choices=["batch", "running"], default="batch",
                    help="batch = reference semantics (model(x, training=True)); running = standard MC Dropout")
    ap.add_argument("--output_plot_dir", type=str, default="./uq_plots_patient/mc_dropout_no_pool")
    ap.add_argument("--output_csv_dir", type=str, default="./uq_results_patient_no_pool")
    a = ap.parse_args(argv)
    from ..models.cnn import load_model
    from ..uq.drivers import evaluate_mc_dropout

    np.random.seed(a.seed)
    Xu, yu, pids, Xr, yr = _load_test(a.data_dir)
    model = load_model(a.model_path)
    det = model.predict(Xu)
    print(f"Deterministic Accuracy (training=False) on Unbalanced Set: {np.mean((det.ravel() > 0.5) == yu):.4f}")
    res = {}
    res["unbalanced"] = evaluate_mc_dropout(model, Xu, yu, None if global_mode else pids,
                                            "CNN_MCD_Unbalanced", not global_mode, a.n_passes, a.n_bootstrap, a.seed,
                                            a.bn_mode, a.output_csv_dir, a.output_plot_dir,
                                            raw_pred_path="./mc_raw_pred0205.npy" if global_mode else None,
                                            make_plots=not a.no_plots)
    res["balanced"] = evaluate_mc_dropout(model, Xr, yr, None, "CNN_MCD_Balanced_RUS", False, a.n_passes, a.n_bootstrap,
                                          a.seed, a.bn_mode, a.output_csv_dir, a.output_plot_dir, raw_pred_path="",
                                          make_plots=not a.no_plots)
    return res


def evaluate_mcd_global(argv=None):
    return analyze_mcd_patient_level(argv, global_mode=True)


def analyze_de_patient_level(argv=None):
    ap = argparse.ArgumentParser(description="Deep Ensemble UQ evaluation with per-window results.")
    _uq_common(ap)
    ap.add_argument("--model_dir", type=str, default="./models/ensemble_cnn_no_pool")
    ap.add_argument("--pattern", type=str, default="AlCNN_smote_seed{}.keras")
    ap.add_argument("--num_members", type=int, default=5)
    ap.add_argument("--offset", type=int, default=5, help="file index of member 0 (reference loader uses i+5)")
    ap.add_argument("--output_plot_dir", type=str, default="./uq_plots_patient/deep_ensemble_no_pool")
    ap.add_argument("--output_csv_dir", type=str, default="./uq_results_patient_DE_new")
    a = ap.parse_args(argv)
    from ..parallel.ensemble import load_ensemble
    from ..uq.drivers import evaluate_deep_ensemble

    np.random.seed(a.seed)
    Xu, yu, pids, Xr, yr = _load_test(a.data_dir)
    models = load_ensemble(a.model_dir, a.pattern, a.num_members, a.offset)
    return {"unbalanced": evaluate_deep_ensemble(models, Xu, yu, pids, "CNN_DE_Unbalanced", True, a.n_bootstrap, a.seed,
                                                 a.output_csv_dir, a.output_plot_dir, make_plots=not a.no_plots),
            "balanced": evaluate_deep_ensemble(models, Xr, yr, None, "CNN_DE_Balanced_RUS", False, a.n_bootstrap, a.seed,
                                               a.output_csv_dir, a.output_plot_dir, make_plots=not a.no_plots)}


def evaluate_de_global(argv=None):
    ap = argparse.ArgumentParser(description="Deep Ensemble global UQ evaluation (M=20 by default).")
    _uq_common(ap)
    ap.add_argument("--model_prefix", type=str, default="./models/ensemble_cnn/AlCNN_smote_seed")
    ap.add_argument("--num_models", type=int, default=20)
    ap.add_argument("--output_plot_dir", type=str, default="./uq_plots/deep_ensemble20")
    a = ap.parse_args(argv)
    from ..parallel.ensemble import load_ensemble_prefix
    from ..uq.drivers import evaluate_deep_ensemble

    Xu, yu, _, Xr, yr = _load_test(a.data_dir)
    models = load_ensemble_prefix(a.model_prefix, a.num_models)
    return {"unbalanced": evaluate_deep_ensemble(models, Xu, yu, None, "CNN_DE_Unbalanced", False, a.n_bootstrap, a.seed,
                                                 output_plot_dir=a.output_plot_dir, make_plots=not a.no_plots),
            "balanced": evaluate_deep_ensemble(models, Xr, yr, None, "CNN_DE_Balanced_RUS", False, a.n_bootstrap, a.seed,
                                               output_plot_dir=a.output_plot_dir, make_plots=not a.no_plots)}


def aggregate_patient_uq_metrics(argv=None):
    ap = argparse.ArgumentParser(description="Patient-level aggregation of per-window UQ results.")
    ap.add_argument("--input_csv", type=str, default="./detail_patient_MCD.csv")
    ap.add_argument("--output_dir", type=str, default="./patient_level_uq_analysis_MCD")
    ap.add_argument("--tag", type=str, default="MCD")
    a = ap.parse_args(argv)
    from ..analysis.patient import aggregate_patient_uq_metrics as f

    return f(a.input_csv, a.output_dir, a.tag)


def analyze_window_level_uncertainty(argv=None):
    ap = argparse.ArgumentParser(description="Window-level uncertainty vs correctness (binned accuracy).")
    ap.add_argument("--input_csv", type=str, default="./detail_patient_DE.csv")
    ap.add_argument("--num_bins", type=int, default=10)
    a = ap.parse_args(argv)
    from ..analysis.patient import window_level_binning

    return window_level_binning(a.input_csv, num_bins=a.num_bins)


def final_plot_uq_overview_figures(argv=None):
    ap = argparse.ArgumentParser(description="Thesis overview figures (MCD vs DE).")
    ap.add_argument("--mcd_detail", default="./detail_patient_MCD.csv")
    ap.add_argument("--de_detail", default="./detail_patient_DE.csv")
    ap.add_argument("--mcd_summary", default="./patient_level_uq_analysis_MCD/patient_summary_metrics_MCD.csv")
    ap.add_argument("--de_summary", default="./patient_level_uq_analysis_DE/patient_summary_metrics_DE.csv")
    ap.add_argument("--output_dir", default="./final_thesis_plots")
    a = ap.parse_args(argv)
    import pandas as pd

    from ..analysis.figures import final_overview_figures

    ld = lambda p: pd.read_csv(p) if os.path.exists(p) else None  # noqa: E731
    return final_overview_figures(ld(a.mcd_detail), ld(a.de_detail), ld(a.mcd_summary), ld(a.de_summary), a.output_dir)


def patient_accuracy_entropy_correlation(argv=None):
    ap = argparse.ArgumentParser(description="Pearson correlation of patient mean entropy vs accuracy.")
    ap.add_argument("--mcd_csv", default="./patient_level_uq_analysis_MCD/patient_summary_metrics_MCD.csv")
    ap.add_argument("--de_csv", default="./patient_level_uq_analysis_DE/patient_summary_metrics_DE.csv")
    a = ap.parse_args(argv)
    from ..analysis.stats import patient_correlation

    out = {}
    for name, p in (("MC Dropout", a.mcd_csv), ("Deep Ensemble", a.de_csv)):
        if os.path.exists(p):
            out[name] = patient_correlation(p, name)
        else:
            print(f"ERROR: File not found - {p}")
    return out


def window_uncertainty_vs_correctness_mannwhitney(argv=None):
    ap = argparse.ArgumentParser(description="One-sided Mann-Whitney U: entropy of incorrect > correct windows.")
    ap.add_argument("--input_csv", default="./detail_patient_DE.csv")
    ap.add_argument("--method", default="Deep Ensembles")
    a = ap.parse_args(argv)
    from ..analysis.stats import entropy_mannwhitney

    return entropy_mannwhitney(a.input_csv, a.method)


def hyperparameter_plot_mcd_or_de_pass_convergence(argv=None):
    ap = argparse.ArgumentParser(description="Plot overall mean variance convergence vs passes/members.")
    ap.add_argument("--input_csv", type=str, default="")
    ap.add_argument("--output_plot", type=str, default="variance_convergence_plot.png")
    ap.add_argument("--method", type=str, default="mcd", choices=["mcd", "de"])
    a = ap.parse_args(argv)
    if not a.input_csv:
        print("ERROR: --input_csv is required")
        return None
    from ..analysis.figures import plot_variance_convergence

    return plot_variance_convergence(a.input_csv, a.output_plot, a.method)


def convergence_sweep(argv=None):
    ap = argparse.ArgumentParser(description="Compute the variance-convergence CSV for MCD passes or DE members.")
    ap.add_argument("--method", choices=["mcd", "de"], default="mcd")
    ap.add_argument("--data_dir", default="./processed_datasets")
    ap.add_argument("--model_path", default="./AlCNN1D_no_pool.keras")
    ap.add_argument("--model_dir", default="./models/ensemble_cnn_no_pool")
    ap.add_argument("--pattern", default="AlCNN_smote_seed{}.keras")
    ap.add_argument("--offset", type=int, default=5)
    ap.add_argument("--counts", default="5,10,20,30,40,50")
    ap.add_argument("--bn_mode", choices=["batch", "running"], default="running")
    ap.add_argument("--output_csv", default="./convergence_mcd.csv")
    a = ap.parse_args(argv)
    from ..uq import uq_techniques as U
    from ..uq.drivers import convergence_sweep as sweep

    Xu, yu, _, Xr, yr = _load_test(a.data_dir)
    counts = [int(c) for c in a.counts.split(",")]
    if a.method == "mcd":
        from ..models.cnn import load_model

        m = load_model(a.model_path)
        fn = lambda X, n: U.mc_dropout_predict(m, X, n, bn_mode=a.bn_mode)  # noqa: E731
    else:
        from ..parallel.ensemble import load_ensemble

        models = load_ensemble(a.model_dir, a.pattern, max(counts), a.offset)
        fn = lambda X, n: U.deep_ensembles_predict(models[:n], X)  # noqa: E731
    return sweep(fn, counts, Xu, yu, Xr, yr, a.output_csv)


def shhs_cohort_analysis(argv=None):
    from ..data.cohort import main_cohort

    main_cohort(argv)


def shhs_signal_quality(argv=None):
    from ..data.cohort import main_quality

    main_quality(argv)


def uq_demo(argv=None):
    ap = argparse.ArgumentParser(description="Synthetic UQ evaluation demo (uq_techniques.py __main__).")
    ap.add_argument("--output_plot_dir", default="./dummy_uq_plots")
    a = ap.parse_args(argv)
    from ..uq.uq_techniques import demo

    return demo(a.output_plot_dir)


COMMANDS = {name: fn for name, fn in globals().items()
            if callable(fn) and not name.startswith("_") and name not in ("main",) and fn.__module__ == __name__}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help") or argv[0] not in COMMANDS:
        print("usage: python -m uncertaintyquantification_sleepapnea_1dcnn_amd <command> [flags]\ncommands:\n  " +
              "\n  ".join(sorted(COMMANDS)))
        return 0 if (argv and argv[0] in ("-h", "--help")) else (2 if argv else 0)
    COMMANDS[argv[0]](argv[1:])
    return 0
