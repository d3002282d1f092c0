"""Checkpoint format: the 38 Keras-ordered weight arrays + a JSON architecture config.

The reference persists models as Keras ``.keras`` archives (``cnn_baseline_train.py:230``,
``train_deep_ensemble_cnns.py:170``).  This framework writes a ``.npz`` holding exactly the
arrays ``model.get_weights()`` returns, keyed by their Keras variable names
(``conv1d_1/kernel`` ...), plus ``__config__`` (JSON: ModelSpec, name, optional training state).
Loading uses ``np.load(allow_pickle=False)``: nothing in a checkpoint is ever executed.

Optional Adam state (``__opt__/m/<name>``, ``__opt__/v/<name>``, ``__opt__/step``) allows
mid-training resume.  Paths ending in ``.keras`` are accepted and written as npz content (the
name is kept so the reference's file naming schemes still resolve).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..models.spec import ModelSpec

CONFIG_KEY = "__config__"


def save_weights(path: str, spec: ModelSpec, arrays: List[np.ndarray], name: str = "Alarcon_1D_CNN_Model",
                 extra: Optional[dict] = None, opt_state: Optional[Dict[str, np.ndarray]] = None) -> str:
    names = spec.weight_names()
    if len(arrays) != len(names):
        raise ValueError(f"expected {len(names)} arrays, got {len(arrays)}")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    payload = {n: np.asarray(a, dtype=np.float32) for n, a in zip(names, arrays)}
    cfg = {"spec": spec.to_dict(), "name": name, "format": "apneauq-npz-v1", "weight_names": names}
    if extra:
        cfg["extra"] = extra
    payload[CONFIG_KEY] = np.frombuffer(json.dumps(cfg).encode(), dtype=np.uint8)
    if opt_state:
        for k, v in opt_state.items():
            payload[f"__opt__/{k}"] = np.asarray(v)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        np.savez(f, **payload)
    os.replace(tmp, path)
    return path


def load_weights(path: str) -> Tuple[ModelSpec, List[np.ndarray], dict, Dict[str, np.ndarray]]:
    with np.load(path, allow_pickle=False) as z:
        cfg = json.loads(bytes(z[CONFIG_KEY]).decode())
        spec = ModelSpec.from_dict(cfg["spec"])
        arrays = [np.array(z[n], dtype=np.float32) for n in spec.weight_names()]
        opt = {k[len("__opt__/"):]: np.array(z[k]) for k in z.files if k.startswith("__opt__/")}
    return spec, arrays, cfg, opt


def is_checkpoint(path: str) -> bool:
    try:
        with np.load(path, allow_pickle=False) as z:
            return CONFIG_KEY in z.files
    except Exception:
        return False
