"""Baseline training experiment (``models/cnn_baseline_train.py:109-324``).

Load the processed ``.npy`` sets (any of the reference's naming schemes), validate shapes, build
the Alarcón CNN, ``fit`` with EarlyStopping(val_loss, patience, restore_best_weights) and a 10 %
tail validation split, save the checkpoint, evaluate on the unbalanced and RUS test sets.
Unlike the reference (``exit()`` on bad data) errors raise exceptions.
"""
from __future__ import annotations

import argparse
import os
from typing import Dict

import numpy as np
import torch

from ..data.prepare import load_processed
from ..evaluation.evaluate_classification import evaluate_classification_model
from ..models.cnn import al_1d_cnn_create_model
from .callbacks import EarlyStopping

SEED = 2025
PROCESSED_DATA_DIR = "./final_processed_datasets"
MODEL_SAVE_PATH = "./alarcon_cnn_model.keras"
NUM_EPOCHS = 30
BATCH_SIZE = 1024
EARLY_STOPPING_PATIENCE = 5


def run_cnn_experiment(data_dir: str = PROCESSED_DATA_DIR, model_save_path: str = MODEL_SAVE_PATH,
                       num_epochs: int = NUM_EPOCHS, batch_size: int = BATCH_SIZE, seed: int = SEED,
                       early_stopping_patience: int = EARLY_STOPPING_PATIENCE, device=None,
                       verbose: int = 2) -> Dict:
    print("--- Starting 1D CNN Model Experiment ---")
    np.random.seed(seed)
    torch.manual_seed(seed)
    Xtr = load_processed(data_dir, "X_train_win_std_smote.npy")
    ytr = load_processed(data_dir, "y_train_smote.npy")
    Xub = load_processed(data_dir, "X_test_win_std_unbalanced.npy")
    yub = load_processed(data_dir, "y_test_unbalanced.npy")
    try:
        Xrus = load_processed(data_dir, "X_test_win_std_rus.npy")
        yrus = load_processed(data_dir, "y_test_rus.npy")
    except FileNotFoundError:
        Xrus = yrus = None
    if Xtr.ndim != 3:
        raise ValueError(f"Expected X_train shape like (samples, time_steps, features), got {Xtr.shape}")
    if Xtr.size == 0 or Xub.size == 0:
        raise ValueError("One or more loaded datasets are empty.")
    shape = (Xtr.shape[1], Xtr.shape[2])
    model = al_1d_cnn_create_model(shape, seed=seed, device=device)
    model.summary()
    es = EarlyStopping(monitor="val_loss", patience=early_stopping_patience, restore_best_weights=True)
    hist = model.fit(Xtr, ytr.astype(np.float32), epochs=num_epochs, batch_size=batch_size, validation_split=0.1,
                     callbacks=[es], verbose=verbose)
    d = os.path.dirname(model_save_path)
    if d:
        os.makedirs(d, exist_ok=True)
    model.save(model_save_path)
    print(f"Model saved successfully to '{model_save_path}'.")
    out = {"history": hist.history, "model_path": model_save_path}
    out["unbalanced"] = evaluate_classification_model(model, Xub, yub, "CNN - Unbalanced Test Set")
    if Xrus is not None and Xrus.size:
        out["rus"] = evaluate_classification_model(model, Xrus, yrus, "CNN - Balanced Test Set (RUS)")
    print("--- 1D CNN Model Experiment Script Finished ---")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="Train, save, and evaluate a 1D CNN model on processed time-series data.")
    ap.add_argument("--data_dir", type=str, default=PROCESSED_DATA_DIR)
    ap.add_argument("--model_save_path", type=str, default=MODEL_SAVE_PATH)
    ap.add_argument("--epochs", type=int, default=NUM_EPOCHS)
    ap.add_argument("--batch_size", type=int, default=BATCH_SIZE)
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--early_stopping_patience", type=int, default=EARLY_STOPPING_PATIENCE)
    a = ap.parse_args(argv)
    run_cnn_experiment(a.data_dir, a.model_save_path, a.epochs, a.batch_size, a.seed, a.early_stopping_patience)


if __name__ == "__main__":
    main()
