"""Every public function of the reference's scripts is importable under its reference name from the
matching ``cli`` module and behaves like the reference on edge cases."""
import numpy as np
import pandas as pd
import pytest
import torch
from scipy.stats import pearsonr

REF_FUNCS = {
    "evaluate_de_global": ["load_ensemble", "evaluate_ensemble"],
    "evaluate_mcd_global": ["evaluate_mc_dropout"],
    "analyze_mcd_patient_level": ["evaluate_mc_dropout"],
    "analyze_de_patient_level": ["load_ensemble", "evaluate_deep_ensemble"],
    "patient_accuracy_entropy_correlation": ["calculate_and_print_correlation"],
    "final_plot_uq_overview_figures": ["load_data"],
    "cnn_baseline_train": ["al_1d_cnn_create_model", "run_cnn_experiment"],
    "train_deep_ensemble_cnns": ["al_1d_cnn_create_model", "train_ensemble"],
    "shhs_signal_quality": ["analyze_signal_quality"],
    "shhs_cohort_analysis": ["analyze_cohort"],
    "hyperparameter_plot_mcd_or_de_pass_convergence": ["plot_variance_convergence"],
    "preprocess_shhs_raw": ["check_artifacts_and_missing_values", "calculate_sleep_time", "remove_artifacts",
                            "get_edf_channels", "resample_signals", "parse_xml_annotations",
                            "segment_and_label_edf_data", "process_single_file", "process_all_files", "main"],
    "prepare_numpy_datasets": ["reshape_flat_to_3d", "standardize_per_window", "prepare_final_datasets"],
}


@pytest.mark.parametrize("module", list(REF_FUNCS))
def test_reference_names_exported(module):
    import importlib

    m = importlib.import_module(f"uncertaintyquantification_sleepapnea_1dcnn_amd.cli.{module}")
    for f in REF_FUNCS[module]:
        assert callable(getattr(m, f)), (module, f)


def test_correlation_and_load_data(tmp_path):
    from uncertaintyquantification_sleepapnea_1dcnn_amd.cli.final_plot_uq_overview_figures import load_data
    from uncertaintyquantification_sleepapnea_1dcnn_amd.cli.patient_accuracy_entropy_correlation import (
        calculate_and_print_correlation)

    rng = np.random.default_rng(0)
    df = pd.DataFrame({"mean_entropy": rng.random(30), "patient_accuracy": rng.random(30)})
    df.loc[3, "mean_entropy"] = np.nan
    p = tmp_path / "summary.csv"
    df.to_csv(p, index=False)
    r, pv = calculate_and_print_correlation(str(p), "MC Dropout", "mean_entropy", "patient_accuracy")
    clean = df.dropna()
    er, ep = pearsonr(clean["mean_entropy"], clean["patient_accuracy"])
    assert abs(r - er) < 1e-12 and abs(pv - ep) < 1e-12
    assert calculate_and_print_correlation(str(tmp_path / "missing.csv"), "DE", "mean_entropy",
                                           "patient_accuracy") == (None, None)
    assert load_data(str(tmp_path / "missing.csv")) is None
    assert load_data(str(p)).shape == df.shape


def test_global_drivers_reference_signatures():
    from uncertaintyquantification_sleepapnea_1dcnn_amd.cli.evaluate_de_global import evaluate_ensemble
    from uncertaintyquantification_sleepapnea_1dcnn_amd.cli.evaluate_mcd_global import evaluate_mc_dropout
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D

    g = torch.Generator().manual_seed(0)
    x = torch.randn(40, 60, 4, generator=g).numpy()
    y = (np.arange(40) % 3 == 0).astype(int)
    models = [AlarconCNN1D(seed=i, device="cpu") for i in range(2)]
    assert evaluate_ensemble(models, x.reshape(40, -1), y, "bad") is None  # 2-D input rejected (:48-50)
    de = evaluate_ensemble(models, x, y, "DE_test", n_bootstrap=5, make_plots=False)
    mcd = evaluate_mc_dropout(models[0], x, y, "MCD_test", n_passes=3, n_bootstrap=5, make_plots=False)
    for res in (de, mcd):
        assert "mean_predictive_variance" in res or any("variance" in k for k in res)
        assert sum(k.endswith("_ci_lower") for k in res) == 6


def test_mc_dropout_running_calls_draw_fresh_masks():
    """Like model(x, training=True), consecutive mc_dropout_predict calls differ."""
    import numpy as np

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

    m = AlarconCNN1D(seed=3, device="cpu")
    x = np.random.default_rng(0).standard_normal((6, 60, 4)).astype(np.float32)
    a = U.mc_dropout_predict(m, x, n_pred=2, bn_mode="running")
    b = U.mc_dropout_predict(m, x, n_pred=2, bn_mode="running")
    assert a.shape == b.shape == (2, 6, 1)
    assert not np.array_equal(a, b)
    assert m._call_counter == 4
