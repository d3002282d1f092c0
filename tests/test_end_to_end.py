"""End-to-end synthetic pipeline (SURVEY §4 test 6): EDF/XML -> CSV -> .npy -> train -> MCD & DE UQ
-> per-window CSV schema -> patient aggregation / binning / statistics / figures, via the CLI."""
import os

import numpy as np
import pandas as pd

from uncertaintyquantification_sleepapnea_1dcnn_amd.cli import commands as C
from uncertaintyquantification_sleepapnea_1dcnn_amd.data import synthetic
from uncertaintyquantification_sleepapnea_1dcnn_amd.uq.drivers import DETAIL_COLUMNS


def test_pipeline(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    for i in range(5):
        synthetic.write_synthetic_recording("edf", "xml", f"20{i:04d}", hours=5.05, seed=i, n_events=60)
    C.preprocess_shhs_raw(["--edf_folder", "edf", "--xml_folder", "xml", "--output_csv", "all.csv"])
    df = pd.read_csv("all.csv")
    assert df.shape[1] == 244 and df["Patient_ID"].nunique() == 5
    C.prepare_numpy_datasets(["--input_csv", "all.csv", "--output_dir", "proc", "--test_size", "0.4"])
    C.cnn_baseline_train(["--data_dir", "proc", "--model_save_path", "AlCNN1D_no_pool.keras", "--epochs", "1",
                          "--batch_size", "256"])
    assert os.path.exists("AlCNN1D_no_pool.keras")
    C.train_deep_ensemble_cnns(["--data_dir", "proc", "--num_models", "2", "--epochs", "1", "--batch_size", "256",
                                "--save_dir", "ens", "--name_offset", "5"])
    res = C.analyze_mcd_patient_level(["--data_dir", "proc", "--n_passes", "4", "--n_bootstrap", "5", "--no_plots",
                                       "--output_csv_dir", "csv"])
    assert len(res["unbalanced"]) == 25
    C.analyze_de_patient_level(["--data_dir", "proc", "--model_dir", "ens", "--num_members", "2", "--n_bootstrap", "5",
                                "--no_plots", "--output_csv_dir", "csv"])
    mcd = pd.read_csv("csv/detailed_results_CNN_MCD_Unbalanced.csv")
    de = pd.read_csv("csv/detailed_results_CNN_DE_Unbalanced.csv")
    assert list(mcd.columns) == DETAIL_COLUMNS and list(de.columns) == DETAIL_COLUMNS
    assert np.load("mc_raw_pred0505_CNN_MCD_Unbalanced.npy").shape == (4, len(mcd), 1)
    s1 = C.aggregate_patient_uq_metrics(["--input_csv", "csv/detailed_results_CNN_MCD_Unbalanced.csv",
                                         "--output_dir", "pm", "--tag", "MCD"])
    s2 = C.aggregate_patient_uq_metrics(["--input_csv", "csv/detailed_results_CNN_DE_Unbalanced.csv",
                                         "--output_dir", "pd", "--tag", "DE"])
    assert list(s1.columns) == ["Patient_ID", "mean_variance", "median_variance", "std_variance", "mean_entropy",
                                "median_entropy", "std_entropy", "patient_accuracy", "num_windows"]
    b = C.analyze_window_level_uncertainty(["--input_csv", "csv/detailed_results_CNN_DE_Unbalanced.csv"])
    assert int(b["window_count"].sum()) == len(de)
    C.patient_accuracy_entropy_correlation(["--mcd_csv", "pm/patient_summary_metrics_MCD.csv",
                                            "--de_csv", "pd/patient_summary_metrics_DE.csv"])
    C.window_uncertainty_vs_correctness_mannwhitney(["--input_csv", "csv/detailed_results_CNN_MCD_Unbalanced.csv",
                                                     "--method", "MC Dropout"])
    figs = C.final_plot_uq_overview_figures(["--mcd_detail", "csv/detailed_results_CNN_MCD_Unbalanced.csv",
                                             "--de_detail", "csv/detailed_results_CNN_DE_Unbalanced.csv",
                                             "--mcd_summary", "pm/patient_summary_metrics_MCD.csv",
                                             "--de_summary", "pd/patient_summary_metrics_DE.csv", "--output_dir", "figs"])
    assert len(figs) == 4 and all(os.path.exists(f) for f in figs)
    import shutil

    for i, src in enumerate(["ens/AlCNN_smote_seed5.keras", "ens/AlCNN_smote_seed6.keras"]):
        shutil.copy(src, f"ens/glob{i}.keras")  # evaluate_de_global.py naming: {prefix}{i}.keras
    g = C.evaluate_de_global(["--data_dir", "proc", "--model_prefix", "ens/glob", "--num_models", "2", "--n_bootstrap", "3",
                              "--no_plots"])
    assert len(g["unbalanced"]) == 25 and len(g["balanced"]) == 25
    C.convergence_sweep(["--method", "de", "--data_dir", "proc", "--model_dir", "ens", "--counts", "1,2",
                         "--output_csv", "conv.csv"])
    assert C.hyperparameter_plot_mcd_or_de_pass_convergence(["--input_csv", "conv.csv", "--method", "de",
                                                             "--output_plot", "conv.png"]) == "conv.png"
