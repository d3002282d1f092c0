"""Synthetic SHHS2-shaped data (no dataset download is possible or needed).

* :func:`synthetic_windows` — standardised (N, L, C) windows with a learnable apnea signature
  (SaO2 desaturation + reduced effort amplitude in positive windows), labels, patient ids.
* :func:`write_synthetic_recording` — a full-night EDF (SaO2/PR at 1 Hz, effort belts at 10 Hz)
  plus its NSRR XML with obstructive apnea / hypopnea events, for end-to-end pipeline tests.
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

import numpy as np

from .annotations import write_xml_annotations
from .edf import write_edf


def synthetic_windows(n: int, length: int = 60, channels: int = 4, pos_frac: float = 0.3, seed: int = 0,
                      n_patients: int = 50, standardize: bool = True) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    rs = np.random.RandomState(seed)
    y = (rs.rand(n) < pos_frac).astype(np.int64)
    t = np.arange(length)[None, :]
    x = rs.randn(n, length, channels).astype(np.float64) * 0.5
    phase = rs.rand(n, 1) * 2 * np.pi
    for c in range(min(channels, 4)):
        x[:, :, c] += np.sin(2 * np.pi * t / (4 + c) + phase)
    # apnea signature: desaturation dip in channel 0, damped effort in channels 2-3
    dip = np.exp(-0.5 * ((t - length * 0.6) / (length * 0.12)) ** 2)
    x[:, :, 0] -= 2.5 * y[:, None] * dip
    if channels > 2:
        x[:, :, 2:] *= (1.0 - 0.6 * y[:, None, None] * (t[..., None] > length * 0.3))
    if standardize:
        x = (x - x.mean(1, keepdims=True)) / (x.std(1, keepdims=True) + 1e-8)
    pids = rs.randint(200000, 200000 + n_patients, size=n)
    return x.astype(np.float32), y, pids


def write_synthetic_recording(edf_dir: str, xml_dir: str, nsrr_id: str, hours: float = 5.5, seed: int = 0,
                              n_events: int = 40, belt_rate: float = 10.0) -> Tuple[str, str, List[Dict]]:
    rs = np.random.RandomState(seed)
    secs = int(hours * 3600)
    t1 = np.arange(secs)
    spo2 = 95 + rs.randn(secs) * 0.8
    pr = 65 + 5 * np.sin(2 * np.pi * t1 / 900) + rs.randn(secs)
    tb = np.arange(int(secs * belt_rate)) / belt_rate
    thor = np.sin(2 * np.pi * tb / 4.0) + rs.randn(tb.size) * 0.1
    abdo = np.sin(2 * np.pi * tb / 4.0 + 0.5) + rs.randn(tb.size) * 0.1
    events = []
    starts = np.sort(rs.choice(np.arange(120, secs - 120, 60), size=n_events, replace=False))
    for s in starts:
        dur = float(rs.randint(10, 40))
        concept = "Obstructive apnea|Obstructive Apnea" if rs.rand() < 0.5 else "Hypopnea|Hypopnea"
        s = float(s + rs.randint(0, 30))
        events.append({"event_type": "Respiratory|Respiratory", "event_concept": concept, "start": s, "duration": dur})
        a, b = int(s), int(s + dur)
        spo2[a + 10: b + 15] -= 4.0
        m = (tb >= a) & (tb < b)
        thor[m] *= 0.2
        abdo[m] *= 0.2
    # a few out-of-range artifacts for the interpolation path
    spo2[rs.choice(secs, 20, replace=False)] = 30.0
    pr[rs.choice(secs, 20, replace=False)] = 250.0
    events.insert(0, {"event_type": "", "event_concept": "Recording Start Time", "start": 0.0, "duration": float(secs)})
    os.makedirs(edf_dir, exist_ok=True)
    os.makedirs(xml_dir, exist_ok=True)
    edf = write_edf(os.path.join(edf_dir, f"shhs2-{nsrr_id}.edf"),
                    {"SaO2": spo2, "PR": pr, "THOR RES": thor, "ABDO RES": abdo},
                    {"SaO2": 1.0, "PR": 1.0, "THOR RES": belt_rate, "ABDO RES": belt_rate},
                    phys_ranges={"SaO2": (0, 100), "PR": (0, 250), "THOR RES": (-3, 3), "ABDO RES": (-3, 3)})
    xml = write_xml_annotations(os.path.join(xml_dir, f"shhs2-{nsrr_id}-nsrr.xml"), events)
    return edf, xml, events
