"""SHHS2 raw preprocessing: EDF + NSRR XML -> 60 s labelled windows -> one CSV.

Behaviour of ``data_prepocessing/preprocess_shhs_raw.py`` (P1-P9 in SURVEY §2.1):

* channels ``SaO2, PR, THOR RES, ABDO RES`` with ``H.R.`` as the alternative name of PR;
* artifact removal: SaO2 outside [80, 100] and PR outside [40, 200] -> NaN -> linear interpolation;
* exclusion if any channel has > 10 % NaN (checked after interpolation, as the reference does);
* recording-duration gate (>= 300 min "Recording Start Time"), with the key-name bug fixed (Q7);
* FFT resampling (``scipy.signal.resample``) to 1 Hz, target length ``int(len * target/orig)``;
* non-overlapping 60 s windows flattened time-major (``SaO2_t0, PR_t0, THOR RES_t0, ABDO RES_t0,
  SaO2_t1, ...``) labelled 1 when an obstructive apnea or hypopnea overlaps the window by >= 10 s,
  plus ``Start_Time, End_Time, Apnea/Hypopnea, Patient_ID``.

The reference labels windows with an O(windows x events) ``iterrows`` loop; here the overlap test
is one vectorised (windows x events) array expression.
"""
from __future__ import annotations

import argparse
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
from scipy.signal import resample

from .annotations import APNEA_EVENTS, calculate_sleep_time, parse_xml_annotations
from .edf import EdfHeader, read_edf

SLEEP_APNEA_CHANNELS = ["SaO2", "PR", "THOR RES", "ABDO RES"]
PR_ALIASES = ["H.R."]
COMBINED_FILE = "./SHHS2_ID_all_60.csv"


def get_edf_channels(file_path: str, channels: Sequence[str]) -> Tuple[Dict[str, np.ndarray], Dict[str, float]]:
    labels = EdfHeader(file_path).labels
    want = []
    for ch in channels:
        if ch in labels:
            want.append(ch)
        elif ch == "PR":
            alt = next((a for a in PR_ALIASES if a in labels), None)
            if alt is not None:
                print(f"PR not found. Using alternative {alt} in EDF file {file_path}")
                want.append(alt)
        else:
            print(f"Channel {ch} not found in {file_path}")
    sigs, rates = read_edf(file_path, want)
    out_s: Dict[str, np.ndarray] = {}
    out_r: Dict[str, float] = {}
    for ch in channels:
        src = ch if ch in sigs else (next((a for a in PR_ALIASES if a in sigs), None) if ch == "PR" else None)
        if src is not None:
            out_s[ch] = sigs[src]
            out_r[ch] = rates[src]
    if "PR" in channels and "PR" not in out_s:
        print(f"Warning: 'PR/H.R. channel is missing in {file_path}.")
    return out_s, out_r


def remove_artifacts(signals: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    ranges = {"SaO2": (80.0, 100.0), "PR": (40.0, 200.0)}
    for ch, sig in signals.items():
        if ch not in ranges:
            continue
        lo, hi = ranges[ch]
        bad = (sig < lo) | (sig > hi)
        if np.any(bad):
            sig = sig.astype(np.float64, copy=True)
            sig[bad] = np.nan
            nan = np.isnan(sig)
            if np.any(~nan):
                sig[nan] = np.interp(np.flatnonzero(nan), np.flatnonzero(~nan), sig[~nan])
            signals[ch] = sig
    return signals


def check_artifacts_and_missing_values(signals: Dict[str, np.ndarray], artifact_threshold: float = 0.1) -> bool:
    for sig in signals.values():
        if len(sig) and np.isnan(sig).sum() / len(sig) > artifact_threshold:
            return False
    return True


def resample_signals(signals: Dict[str, np.ndarray], sampling_rates: Dict[str, float], target_rate: float = 1) -> Dict[str, np.ndarray]:
    return {ch: resample(sig, int(len(sig) * (target_rate / sampling_rates[ch]))) for ch, sig in signals.items()}


def window_labels(starts: np.ndarray, ends: np.ndarray, events: pd.DataFrame, min_overlap: float = 10.0) -> np.ndarray:
    """1 where an apnea/hypopnea event overlaps the window by >= min_overlap seconds."""
    if events is None or len(events) == 0:
        return np.zeros(len(starts), dtype=np.int64)
    ev = events[events["event_concept"].isin(APNEA_EVENTS)]
    if len(ev) == 0:
        return np.zeros(len(starts), dtype=np.int64)
    a = ev["start"].to_numpy(np.float64)
    b = a + ev["duration"].to_numpy(np.float64)
    lab = np.zeros(len(starts), dtype=bool)
    for s in range(0, len(starts), 4096):  # bounded (windows x events) blocks
        ov = np.minimum(ends[s: s + 4096, None], b[None]) - np.maximum(starts[s: s + 4096, None], a[None])
        lab[s: s + 4096] = (ov >= min_overlap).any(axis=1)
    return lab.astype(np.int64)


def feature_columns(channels: Sequence[str], window_size: int = 60) -> List[str]:
    return [f"{c}_t{t}" for t in range(window_size) for c in channels]


def segment_and_label_edf_data(edf_df: pd.DataFrame, xml_annotations_df: pd.DataFrame, patient_id, window_size: int = 60,
                               overlap_size: int = 0) -> pd.DataFrame:
    cols = list(edf_df.columns)
    step = window_size - overlap_size
    n = len(edf_df)
    num_windows = (n - window_size + overlap_size) // step + 1 if n >= window_size else 0
    starts = np.arange(num_windows, dtype=np.int64) * step
    starts = starts[starts + window_size <= n]
    if len(starts) == 0:
        return pd.DataFrame()
    vals = edf_df.to_numpy()
    idx = starts[:, None] + np.arange(window_size)[None]
    flat = vals[idx].reshape(len(starts), window_size * len(cols))  # time-major, C order
    ends = starts + window_size
    labels = window_labels(starts.astype(np.float64), ends.astype(np.float64), xml_annotations_df)
    df = pd.DataFrame(flat, columns=feature_columns(cols, window_size))
    df["Start_Time"] = starts
    df["End_Time"] = ends
    df["Apnea/Hypopnea"] = labels
    df["Patient_ID"] = patient_id
    return df


def process_single_file(edf_file_path: str, xml_file_path: str, patient_id, target_channels=SLEEP_APNEA_CHANNELS,
                        target_rate: float = 1, reference_sleep_gate: bool = False) -> Optional[pd.DataFrame]:
    sigs, rates = get_edf_channels(edf_file_path, target_channels)
    sigs = remove_artifacts(sigs)
    if not check_artifacts_and_missing_values(sigs):
        print(f"Excluded {edf_file_path} due to excessive artifacts or missing values.")
        return None
    events = parse_xml_annotations(xml_file_path)
    if not calculate_sleep_time(events, reference_keys=reference_sleep_gate):
        print(f"Excluded {xml_file_path} due to insufficient sleep time.")
        return None
    res = resample_signals(sigs, rates, target_rate)
    m = min(len(v) for v in res.values()) if res else 0
    edf_df = pd.DataFrame({k: v[:m] for k, v in res.items()})
    return segment_and_label_edf_data(edf_df, pd.DataFrame(events), patient_id)


def process_all_files(edf_folder: str, xml_folder: str, target_channels=SLEEP_APNEA_CHANNELS, target_rate: float = 1,
                      num_files: Optional[int] = None, output_csv: str = COMBINED_FILE,
                      reference_sleep_gate: bool = False) -> Optional[pd.DataFrame]:
    frames = []
    count = 0
    for edf_file in sorted(os.listdir(edf_folder)):
        if num_files is not None and count >= num_files:
            break
        if not edf_file.endswith(".edf"):
            print(f"EDF file for {edf_file} does not have the correct ending. Skipping...")
            continue
        nsrr_id = edf_file.split("-")[1].split(".")[0]
        xml_path = os.path.join(xml_folder, f"shhs2-{nsrr_id}-nsrr.xml")
        edf_path = os.path.join(edf_folder, edf_file)
        if not os.path.exists(xml_path):
            print(f"XML file for {edf_file} not found. Skipping...")
            continue
        print(f"Processing {count}: {edf_path} and {xml_path}")
        try:
            df = process_single_file(edf_path, xml_path, nsrr_id, target_channels, target_rate, reference_sleep_gate)
            if df is not None and len(df):
                frames.append(df)
        except Exception as e:  # per-file fault isolation, as the reference (preprocess_shhs_raw.py:316)
            print(f"Error processing {edf_path} and {xml_path}: {e}")
        count += 1
    if not frames:
        return None
    out = pd.concat(frames, ignore_index=True)
    if output_csv:
        out.to_csv(output_csv, index=False)
        print(f"Saved combined dataset to {output_csv}")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="Process SHHS2 EDF + XML into 60 s labelled windows (CSV).")
    ap.add_argument("--edf_folder", type=str, default="")
    ap.add_argument("--xml_folder", type=str, default="")
    ap.add_argument("--num_files", type=int, default=None, help="Number of files to process")
    ap.add_argument("--output_csv", type=str, default=COMBINED_FILE)
    ap.add_argument("--reference_sleep_gate", action="store_true",
                    help="reproduce the reference's KeyError-based sleep-time gate (excludes every file)")
    a = ap.parse_args(argv)
    process_all_files(a.edf_folder, a.xml_folder, SLEEP_APNEA_CHANNELS, 1, a.num_files, a.output_csv,
                      a.reference_sleep_gate)


if __name__ == "__main__":
    main()
