"""Binary classification evaluation with the reference's metric set and return dictionary.

Equivalent of ``evaluation/evaluate_classification.py:7-153``: predictions from ``model.predict``
(fused HIP inference on the GPU), threshold ``> 0.5``, classification report (text + dict),
ROC-AUC, PR-AUC (``precision_recall_curve`` + trapezoid ``auc``), Cohen's kappa, MCC, the 2x2
confusion matrix (padded when a class is absent), sensitivity and specificity; the same 14 keys.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
from sklearn.metrics import (auc, classification_report, cohen_kappa_score, confusion_matrix, matthews_corrcoef,
                             precision_recall_curve, roc_auc_score)


def classification_metrics(y_test, y_pred_probs, evaluation_description: str = "Evaluation",
                           verbose: bool = True) -> Optional[Dict]:
    y_test = np.asarray(y_test).reshape(-1)
    p = np.asarray(y_pred_probs, dtype=np.float64)
    if p.ndim > 1 and p.shape[1] == 1:
        p = p.reshape(-1)
    y_pred = (p > 0.5).astype(int)
    try:
        report_str = classification_report(y_test, y_pred, labels=[0, 1], target_names=["Normal (0)", "Apnea/Hypopnea (1)"],
                                           zero_division=0)
        report_dict = classification_report(y_test, y_pred, output_dict=True, zero_division=0)
        accuracy = report_dict.get("accuracy", float(np.mean(y_pred == y_test)))
        if len(np.unique(y_test)) < 2:
            roc_auc = auc_pr = np.nan
            if verbose:
                print("Warning: Only one class present in y_test. Skipping ROC AUC and AUC-PR calculation.")
        else:
            yt = y_test.astype(float)
            roc_auc = roc_auc_score(yt, p)
            prec, rec, _ = precision_recall_curve(yt, p)
            auc_pr = auc(rec, prec)
        kappa = cohen_kappa_score(y_test, y_pred)
        mcc = matthews_corrcoef(y_test, y_pred)
        cm = confusion_matrix(y_test, y_pred)
        if cm.shape != (2, 2):
            padded = np.zeros((2, 2), dtype=int)
            padded[: cm.shape[0], : cm.shape[1]] = cm
            cm = padded
        tn, fp, fn, tp = cm.ravel()
        sensitivity = tp / (tp + fn) if (tp + fn) > 0 else 0.0
        specificity = tn / (tn + fp) if (tn + fp) > 0 else 0.0
    except Exception as e:
        print(f"Error calculating metrics: {e}")
        return None
    if verbose:
        print(f"\n--- {evaluation_description} ---")
        print(f"\nClassification Report:\n{report_str}")
        print(f"Overall Accuracy: {accuracy:.4f}")
        print(f"ROC AUC: {roc_auc:.4f}" if not np.isnan(roc_auc) else "ROC AUC: N/A (only one class in y_test)")
        print(f"AUC-PR: {auc_pr:.4f}" if not np.isnan(auc_pr) else "AUC-PR: N/A (only one class in y_test)")
        print(f"Cohen's Kappa: {kappa:.4f}")
        print(f"Matthews Correlation Coefficient: {mcc:.4f}")
        print(f"Overall Sensitivity (Recall): {sensitivity:.4f}")
        print(f"Overall Specificity: {specificity:.4f}")
        print(f"Confusion Matrix:\n{cm}")
        print(f"   [[TN={tn}  FP={fp}]")
        print(f"    [FN={fn}  TP={tp}]]")
        print(f"--- Evaluation Complete for {evaluation_description} ---")
    return {
        "evaluation_description": evaluation_description,
        "classification_report_dict": report_dict,
        "accuracy": accuracy,
        "roc_auc": None if np.isnan(roc_auc) else roc_auc,
        "auc_pr": None if np.isnan(auc_pr) else auc_pr,
        "cohen_kappa": kappa,
        "mcc": mcc,
        "overall_sensitivity": sensitivity,
        "overall_specificity": specificity,
        "confusion_matrix": cm,
        "tn": tn, "fp": fp, "fn": fn, "tp": tp,
    }


def evaluate_classification_model(model, X_test, y_test, evaluation_description: str = "Evaluation") -> Optional[Dict]:
    """Predict with ``model.predict`` and compute the metric dictionary (reference signature)."""
    try:
        probs = np.asarray(model.predict(X_test, verbose=0) if hasattr(model, "predict") else model(X_test))
        if probs.ndim > 1 and probs.shape[1] == 1:
            probs = probs.reshape(-1)
    except Exception as e:
        print(f"Error during model prediction: {e}")
        return None
    print(f"\n--- {evaluation_description} ---")
    print("Calculating metrics...")
    return classification_metrics(y_test, probs, evaluation_description)
