"""CSV of flattened windows -> patient-split, per-window standardised, balanced ``.npy`` sets.

Behaviour of ``data_prepocessing/prepare_numpy_datasets.py:99-265``:
NaN features filled with global column means; patient-grouped
``GroupShuffleSplit(n_splits=1, test_size, random_state=seed)`` with an overlap check; (N, 240)
-> (N, 60, 4) C-order reshape; per-window standardisation ``(x - mean_t) / (std_t + 1e-8)``
(population std); SMOTE on the flattened training set (fallback: unbalanced); RUS on the test
set for a balanced copy; files saved under the reference's names.

The standardisation runs on the GPU when one is present (the arrays are then already device
resident for training).  ``load_processed`` resolves the three inconsistent file/dir naming
schemes of the reference so every stage reads what the previous one wrote.
"""
from __future__ import annotations

import argparse
import os
from typing import Dict, Optional

import numpy as np
import pandas as pd
from sklearn.model_selection import GroupShuffleSplit

from .balance import SMOTE, RandomUnderSampler

SHHS2_CSV_ALL = "./SHHS2_ID_all.csv"
OUTPUT_DIR = "./processed_datasets2"
TEST_SIZE = 0.20
RANDOM_SEED = 2025
ORIGINAL_FEATURES = ["SaO2", "PR", "THOR RES", "ABDO RES"]
NUM_FEATURES = len(ORIGINAL_FEATURES)
TIME_STEPS = 60
LABEL_COL = "Apnea/Hypopnea"
GROUP_COL = "Patient_ID"
FEATURE_COLS = [f"{c}_t{t}" for t in range(TIME_STEPS) for c in ORIGINAL_FEATURES]

# canonical file name -> legacy aliases used by downstream reference scripts
FILE_ALIASES: Dict[str, tuple] = {
    "X_train_win_std_smote.npy": ("X_train_std_smote.npy",),
    "y_train_smote.npy": (),
    "X_test_win_std_unbalanced.npy": ("X_test_std_unbalanced.npy",),
    "y_test_unbalanced.npy": (),
    "patient_ids_test_unbalanced.npy": (),
    "X_test_win_std_rus.npy": ("X_test_std_rus.npy",),
    "y_test_rus.npy": (),
}


def reshape_flat_to_3d(data_flat: np.ndarray, steps: int = TIME_STEPS, features: int = NUM_FEATURES) -> np.ndarray:
    if data_flat.shape[1] != steps * features:
        raise ValueError(f"Incorrect number of features for reshaping: {data_flat.shape[1]} != {steps * features}")
    return data_flat.reshape((data_flat.shape[0], steps, features))


def standardize_per_window(data_3d, epsilon: float = 1e-8, device: Optional[str] = None) -> np.ndarray:
    """Per-window, per-channel z-score over the time axis (ddof=0), float64 like the reference."""
    if device is None:
        try:
            import torch

            device = "cuda" if torch.cuda.is_available() and np.asarray(data_3d).size > 1_000_000 else "cpu"
        except Exception:
            device = "cpu"
    if device != "cpu":
        import torch

        x = torch.as_tensor(np.asarray(data_3d, np.float64), device=device)
        if x.is_cuda and x.dim() == 3 and x.shape[1] * x.shape[2] * 8 <= 65536 and x.shape[2] <= 256:
            from ..ops import _ext

            _ext.require()  # K14: csrc/prep.hip standardize_kernel (fp64, LDS-staged windows)
            return torch.ops.apneauq.prep_standardize(x, float(epsilon)).cpu().numpy()
        mean = x.mean(dim=1, keepdim=True)
        std = x.std(dim=1, keepdim=True, unbiased=False)
        return ((x - mean) / (std + epsilon)).cpu().numpy()
    mean = np.mean(data_3d, axis=1, keepdims=True)
    std = np.std(data_3d, axis=1, keepdims=True)
    return (data_3d - mean) / (std + epsilon)


def prepare_final_datasets(input_csv: str = SHHS2_CSV_ALL, output_dir: str = OUTPUT_DIR, test_size: float = TEST_SIZE,
                           seed: int = RANDOM_SEED, write_aliases: bool = True) -> Optional[Dict[str, np.ndarray]]:
    print(f"--- Starting Final Data Preparation (Window-Level Standardization) ---")
    os.makedirs(output_dir, exist_ok=True)
    try:
        full = pd.read_csv(input_csv)
        if not all(c in full.columns for c in FEATURE_COLS + [LABEL_COL, GROUP_COL]):
            raise ValueError("Missing required columns in input CSV.")
    except FileNotFoundError:
        print(f"ERROR: Input CSV file not found at {input_csv}")
        return None
    except Exception as e:
        print(f"ERROR: Failed to load or validate CSV: {e}")
        return None
    if full[FEATURE_COLS].isnull().values.any():
        print("NaN values found! Filling with global column means.")
        full[FEATURE_COLS] = full[FEATURE_COLS].fillna(full[FEATURE_COLS].mean())
    X_flat, y, groups = full[FEATURE_COLS], full[LABEL_COL], full[GROUP_COL]
    splitter = GroupShuffleSplit(n_splits=1, test_size=test_size, random_state=seed)
    train_idx, test_idx = next(splitter.split(X_flat, y, groups))
    y_train, y_test = y.iloc[train_idx], y.iloc[test_idx]
    g_train, g_test = groups.iloc[train_idx], groups.iloc[test_idx]
    if set(g_train.unique()) & set(g_test.unique()):
        print("WARNING: Patient overlap detected between train and test sets!")
    else:
        print("Patient split verified: No overlap.")
    X_train = standardize_per_window(reshape_flat_to_3d(X_flat.iloc[train_idx].values))
    X_test = standardize_per_window(reshape_flat_to_3d(X_flat.iloc[test_idx].values))
    n_tr, steps, feats = X_train.shape
    try:
        Xs, ys = SMOTE(random_state=seed).fit_resample(X_train.reshape(n_tr, steps * feats), y_train)
        X_train_smote, y_train_smote = reshape_flat_to_3d(Xs, steps, feats), np.asarray(ys)
        print(f"SMOTE balanced train shape: {X_train_smote.shape}")
    except Exception as e:
        print(f"ERROR during SMOTE: {e}. Using original window-standardized training data.")
        X_train_smote, y_train_smote = X_train.copy(), y_train.values.copy()
    X_rus = y_rus = None
    try:
        Xr, yr = RandomUnderSampler(random_state=seed).fit_resample(X_test.reshape(X_test.shape[0], steps * feats), y_test)
        X_rus, y_rus = reshape_flat_to_3d(Xr, steps, feats), np.asarray(yr)
    except Exception as e:
        print(f"ERROR during RUS: {e}. Skipping RUS balancing for balanced test set.")
    out = {"X_train_win_std_smote.npy": X_train_smote, "y_train_smote.npy": y_train_smote,
           "X_test_win_std_unbalanced.npy": X_test, "y_test_unbalanced.npy": y_test.values,
           "patient_ids_test_unbalanced.npy": g_test.values}
    if X_rus is not None:
        out["X_test_win_std_rus.npy"] = X_rus
        out["y_test_rus.npy"] = y_rus
    for name, arr in out.items():
        np.save(os.path.join(output_dir, name), arr)
        if write_aliases:
            for alias in FILE_ALIASES.get(name, ()):
                np.save(os.path.join(output_dir, alias), arr)
    print("Datasets saved successfully.")
    return out


def load_processed(data_dir: str, name: str, mmap: bool = False) -> np.ndarray:
    """Load a processed array by canonical name, falling back to legacy aliases."""
    cands = [name] + list(FILE_ALIASES.get(name, ()))
    for k, v in FILE_ALIASES.items():
        if name in v:
            cands = [k] + list(v)
    for c in cands:
        p = os.path.join(data_dir, c)
        if os.path.exists(p):
            return np.load(p, mmap_mode="r" if mmap else None, allow_pickle=False)
    raise FileNotFoundError(f"none of {cands} found in {data_dir}")


def main(argv=None):
    ap = argparse.ArgumentParser(description="Prepare final datasets for ML with window-level standardization.")
    ap.add_argument("--input_csv", type=str, default=SHHS2_CSV_ALL)
    ap.add_argument("--output_dir", type=str, default=OUTPUT_DIR)
    ap.add_argument("--test_size", type=float, default=TEST_SIZE)
    ap.add_argument("--seed", type=int, default=RANDOM_SEED)
    a = ap.parse_args(argv)
    prepare_final_datasets(a.input_csv, a.output_dir, a.test_size, a.seed)


if __name__ == "__main__":
    main()
