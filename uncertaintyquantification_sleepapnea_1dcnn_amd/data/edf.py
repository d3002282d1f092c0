"""Minimal EDF/EDF+ reader and writer (pyedflib is not available; none is needed).

Replaces ``pyedflib.EdfReader`` as used by ``data_prepocessing/preprocess_shhs_raw.py:128-155``:
per-channel physical signals (digital int16 -> physical via the header's linear map) and
sampling rates (samples per record / record duration).  The whole data section is decoded with
one vectorised NumPy pass per signal (no per-record Python loop).  ``write_edf`` produces valid
EDF files; the test suite uses it to build synthetic SHHS2-like recordings.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


def _field(b: bytes, n: int, off: int) -> Tuple[str, int]:
    return b[off: off + n].decode("latin1").strip(), off + n


class EdfHeader:
    def __init__(self, path: str):
        with open(path, "rb") as f:
            fixed = f.read(256)
            if len(fixed) < 256:
                raise ValueError(f"{path}: not an EDF file (header too short)")
            off = 0
            self.version, off = _field(fixed, 8, off)
            self.patient, off = _field(fixed, 80, off)
            self.recording, off = _field(fixed, 80, off)
            self.startdate, off = _field(fixed, 8, off)
            self.starttime, off = _field(fixed, 8, off)
            hb, off = _field(fixed, 8, off)
            self.header_bytes = int(hb)
            self.reserved, off = _field(fixed, 44, off)
            nr, off = _field(fixed, 8, off)
            self.n_records = int(nr)
            dur, off = _field(fixed, 8, off)
            self.record_duration = float(dur)
            ns, off = _field(fixed, 4, off)
            self.n_signals = int(ns)
            sig = f.read(256 * self.n_signals)
        ns = self.n_signals

        def col(width: int, start: int) -> Tuple[List[str], int]:
            vals = [sig[start + i * width: start + (i + 1) * width].decode("latin1").strip() for i in range(ns)]
            return vals, start + width * ns

        o = 0
        self.labels, o = col(16, o)
        self.transducer, o = col(80, o)
        self.phys_dim, o = col(8, o)
        pmin, o = col(8, o)
        pmax, o = col(8, o)
        dmin, o = col(8, o)
        dmax, o = col(8, o)
        self.prefilter, o = col(80, o)
        nsamp, o = col(8, o)
        self.phys_min = np.array([float(v) for v in pmin])
        self.phys_max = np.array([float(v) for v in pmax])
        self.dig_min = np.array([float(v) for v in dmin])
        self.dig_max = np.array([float(v) for v in dmax])
        self.samples_per_record = np.array([int(v) for v in nsamp], dtype=np.int64)
        self.path = path

    def sample_rate(self, i: int) -> float:
        return float(self.samples_per_record[i]) / self.record_duration if self.record_duration else 0.0

    def getSignalLabels(self) -> List[str]:  # pyedflib-compatible name
        return list(self.labels)


def read_edf(path: str, channels: Optional[Sequence[str]] = None) -> Tuple[Dict[str, np.ndarray], Dict[str, float]]:
    """Return ({label: physical float64 signal}, {label: Hz}) for the requested channels."""
    h = EdfHeader(path)
    rec = int(h.samples_per_record.sum())
    n_rec = h.n_records
    raw = np.fromfile(path, dtype="<i2", offset=h.header_bytes)
    if n_rec < 0:
        n_rec = raw.size // rec
    raw = raw[: n_rec * rec].reshape(n_rec, rec)
    starts = np.concatenate([[0], np.cumsum(h.samples_per_record)])
    want = h.labels if channels is None else [c for c in channels if c in h.labels]
    sigs: Dict[str, np.ndarray] = {}
    rates: Dict[str, float] = {}
    for name in want:
        i = h.labels.index(name)
        d = raw[:, starts[i]: starts[i + 1]].reshape(-1).astype(np.float64)
        span_d = h.dig_max[i] - h.dig_min[i]
        gain = (h.phys_max[i] - h.phys_min[i]) / span_d if span_d else 1.0
        sigs[name] = (d - h.dig_min[i]) * gain + h.phys_min[i]
        rates[name] = h.sample_rate(i)
    return sigs, rates


def write_edf(path: str, signals: Dict[str, np.ndarray], rates: Dict[str, float], record_duration: float = 1.0,
              phys_ranges: Optional[Dict[str, Tuple[float, float]]] = None, patient: str = "X", recording: str = "X") -> str:
    """Write signals (physical units) as a 16-bit EDF file."""
    labels = list(signals.keys())
    ns = len(labels)
    spr = [int(round(rates[l] * record_duration)) for l in labels]
    n_rec = min(len(signals[l]) // s for l, s in zip(labels, spr))
    pr = {}
    for l in labels:
        if phys_ranges and l in phys_ranges:
            pr[l] = phys_ranges[l]
        else:
            v = np.asarray(signals[l], np.float64)
            lo, hi = float(np.min(v)), float(np.max(v))
            if hi <= lo:
                hi = lo + 1.0
            pr[l] = (lo, hi)
    dmin, dmax = -32768, 32767

    def f(s: str, n: int) -> bytes:
        return s[:n].ljust(n).encode("latin1")

    hdr = f("0", 8) + f(patient, 80) + f(recording, 80) + f("01.01.01", 8) + f("00.00.00", 8)
    hdr += f(str(256 * (ns + 1)), 8) + f("", 44) + f(str(n_rec), 8) + f(f"{record_duration:g}", 8) + f(str(ns), 4)
    hdr += b"".join(f(l, 16) for l in labels) + b"".join(f("", 80) for _ in labels) + b"".join(f("", 8) for _ in labels)
    hdr += b"".join(f(f"{pr[l][0]:.6g}", 8) for l in labels) + b"".join(f(f"{pr[l][1]:.6g}", 8) for l in labels)
    hdr += b"".join(f(str(dmin), 8) for _ in labels) + b"".join(f(str(dmax), 8) for _ in labels)
    hdr += b"".join(f("", 80) for _ in labels) + b"".join(f(str(s), 8) for s in spr) + b"".join(f("", 32) for _ in labels)
    blocks = []
    for l, s in zip(labels, spr):
        lo, hi = float(f"{pr[l][0]:.6g}"), float(f"{pr[l][1]:.6g}")
        v = np.asarray(signals[l], np.float64)[: n_rec * s]
        d = np.round((v - lo) / (hi - lo) * (dmax - dmin) + dmin)
        blocks.append(np.clip(d, dmin, dmax).astype("<i2").reshape(n_rec, s))
    data = np.concatenate(blocks, axis=1) if blocks else np.zeros((0, 0), "<i2")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as fh:
        fh.write(hdr)
        fh.write(data.tobytes())
    return path
