"""SHHS2 cohort descriptives from the NSRR dataset CSV (``datasets/SHHS_cohort_analysis.py``,
``datasets/SHHS_signal_quality.py``).

Cohort = records with non-missing ``ahi_a0h3a``.  ``analyze_cohort`` reports age (``age_s2``),
gender (1 male / 2 female), race (1 white / 2 black / 3 other) and the AHI distribution with the
clinical severity bins <5, 5-15, 15-30, >=30.  ``analyze_signal_quality`` reports the 1-5 quality
codes of ``quoxim, quhr, quchest, quabdo``.  Both return the computed tables as dicts.
"""
from __future__ import annotations

import argparse
from typing import Dict

import numpy as np
import pandas as pd

AHI, AGE, GENDER, RACE = "ahi_a0h3a", "age_s2", "gender", "race"
QUALITY_VARS = {
    "quoxim": "SaO2 Signal Quality (Oximeter)",
    "quhr": "Heart Rate Signal Quality (Pulse)",
    "quchest": "Thoracic Effort Signal Quality (Chest Inductance)",
    "quabdo": "Abdominal Effort Signal Quality (Abdominal Inductance)",
}
QUALITY_CODES = {1: "<25% artifact-free", 2: "25-49% artifact-free", 3: "50-74% artifact-free",
                 4: "75-94% artifact-free", 5: ">=95% artifact-free"}
AHI_CATEGORIES = ["Normal (AHI < 5.0)", "Mild OSA (AHI 5.0-14.9)", "Moderate OSA (AHI 15.0-29.9)", "Severe OSA (AHI >= 30.0)"]


def _load_cohort(csv_file_path: str) -> pd.DataFrame:
    df = pd.read_csv(csv_file_path, encoding="latin1", low_memory=False)
    if AHI not in df.columns:
        raise KeyError(f"Target AHI column '{AHI}' not found in the dataset")
    return df[df[AHI].notna()].copy()


def ahi_category(v: pd.Series) -> pd.Series:
    v = pd.to_numeric(v, errors="coerce")
    out = np.select([v < 5, (v >= 5) & (v < 15), (v >= 15) & (v < 30), v >= 30], AHI_CATEGORIES, default="Unknown_AHI_Value")
    return pd.Series(out, index=v.index)


def analyze_cohort(csv_file_path: str, verbose: bool = True) -> Dict:
    c = _load_cohort(csv_file_path)
    res: Dict = {"n_cohort": len(c)}
    if AGE in c.columns:
        a = pd.to_numeric(c[AGE], errors="coerce").dropna()
        res["age"] = {"n": len(a), "mean": a.mean(), "std": a.std(), "median": a.median(), "min": a.min(), "max": a.max()}
    for col in (GENDER, RACE):
        if col in c.columns:
            s = c[col].dropna()
            res[col] = {"counts": s.value_counts().sort_index().to_dict(),
                        "percent": (s.value_counts(normalize=True).sort_index() * 100).to_dict()}
    ahi = pd.to_numeric(c[AHI], errors="coerce").dropna()
    res["ahi"] = {"n": len(ahi), "mean": ahi.mean(), "std": ahi.std(), "median": ahi.median(), "min": ahi.min(),
                  "max": ahi.max()}
    cat = ahi_category(c[AHI])
    counts = cat.value_counts().reindex(AHI_CATEGORIES + ["Unknown_AHI_Value"], fill_value=0)
    res["ahi_categories"] = {"counts": counts.to_dict(), "percent": (counts / max(len(cat), 1) * 100).to_dict()}
    if verbose:
        print(f"Analysis cohort defined by non-missing '{AHI}'. N = {res['n_cohort']}")
        if "age" in res:
            a = res["age"]
            print(f"Mean Age: {a['mean']:.1f} ± {a['std']:.1f} years; Median {a['median']:.1f}; Range {a['min']:.1f} - {a['max']:.1f}")
        for col, names in ((GENDER, {1.0: "Male", 2.0: "Female"}), (RACE, {1.0: "White", 2.0: "Black or African American", 3.0: "Other"})):
            if col in res:
                for k, v in res[col]["counts"].items():
                    print(f"  {names.get(k, f'Unknown Code ({k})')} ({k}): {v} ({res[col]['percent'][k]:.1f}%)")
        h = res["ahi"]
        print(f"Mean AHI: {h['mean']:.1f} ± {h['std']:.1f} events/hour; Median {h['median']:.1f}")
        for k in AHI_CATEGORIES:
            print(f"  {k:<25}: {res['ahi_categories']['counts'][k]:<5} ({res['ahi_categories']['percent'][k]:.1f}%)")
    return res


def analyze_signal_quality(csv_file_path: str, verbose: bool = True) -> Dict:
    c = _load_cohort(csv_file_path)
    res: Dict = {"n_cohort": len(c)}
    for col, name in QUALITY_VARS.items():
        if col not in c.columns:
            continue
        s = pd.to_numeric(c[col].dropna(), errors="coerce").dropna()
        counts = s.value_counts().sort_index()
        res[col] = {"name": name, "n_valid": len(s), "n_missing": len(c) - len(s), "mean": s.mean(), "median": s.median(),
                    "std": s.std(), "counts": {int(round(k)): int(v) for k, v in counts.items()},
                    "percent": {int(round(k)): float(v) for k, v in (s.value_counts(normalize=True).sort_index() * 100).items()}}
        if verbose:
            r = res[col]
            print(f"\n--- Statistics for {name} ({col}) ---")
            print(f"N (non-missing values): {r['n_valid']}; missing {r['n_missing']}")
            print(f"Mean score: {r['mean']:.2f}  Median: {r['median']:.2f}  Std: {r['std']:.2f}")
            for k, v in r["counts"].items():
                print(f"  Category {k} ({QUALITY_CODES.get(k, f'Unknown code: {k}')}): {v} ({r['percent'][k]:.1f}%)")
    return res


def main_cohort(argv=None):
    ap = argparse.ArgumentParser(description="Analyze SHHS2 cohort demographics and AHI distribution.")
    ap.add_argument("--csv_file", type=str, default="shhs2-dataset-0.21.0.csv")
    analyze_cohort(ap.parse_args(argv).csv_file)


def main_quality(argv=None):
    ap = argparse.ArgumentParser(description="Analyze SHHS2 signal quality variables.")
    ap.add_argument("--csv_file", type=str, default="shhs2-dataset-0.21.0.csv")
    analyze_signal_quality(ap.parse_args(argv).csv_file)
