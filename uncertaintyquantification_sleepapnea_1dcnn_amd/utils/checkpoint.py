"""Checkpoint formats: the 38 Keras-ordered weight arrays + the architecture.

The reference persists models as Keras ``.keras`` archives (``cnn_baseline_train.py:230``,
``train_deep_ensemble_cnns.py:170``).  The format follows the file name:

* ``*.keras``: a genuine Keras v3 archive (``config.json`` + ``model.weights.h5``, written by
  :mod:`.keras_io` through the pure-Python HDF5 codec), so TF-Keras can open it; run metadata
  and the optional Adam state ride along in an extra ``apneauq_state.npz`` member.
* ``*.h5``: the legacy Keras HDF5 model layout.
* anything else: a ``.npz`` holding exactly the arrays ``model.get_weights()`` returns, keyed by
  their Keras variable names (``conv1d_1/kernel`` ...), plus ``__config__`` (JSON: ModelSpec,
  name, optional training state).

:func:`load_weights` detects the format from the file contents, so ``.keras``/``.h5`` files written
by the reference's own ``model.save`` load too.  Nothing in a checkpoint is ever executed
(``np.load(allow_pickle=False)``, JSON, HDF5 decoded with ``numpy.frombuffer``).

Optional Adam state (``__opt__/m/<name>``, ``__opt__/v/<name>``, ``__opt__/step``) allows
mid-training resume.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..models.spec import ModelSpec
from . import keras_io

CONFIG_KEY = "__config__"


def save_weights(path: str, spec: ModelSpec, arrays: List[np.ndarray], name: str = "Alarcon_1D_CNN_Model",
                 extra: Optional[dict] = None, opt_state: Optional[Dict[str, np.ndarray]] = None) -> str:
    names = spec.weight_names()
    if len(arrays) != len(names):
        raise ValueError(f"expected {len(names)} arrays, got {len(arrays)}")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    if path.endswith(".keras"):
        return keras_io.save(path, spec, arrays, name, extra=extra, opt_state=opt_state)
    if path.endswith(".h5"):
        if opt_state:
            raise ValueError("the legacy .h5 layout carries no optimizer state; use .keras or .npz")
        return keras_io.save_legacy_h5(path, spec, arrays, name)
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
    if keras_io.is_keras_archive(path) or keras_io.is_hdf5(path):
        return keras_io.load(path)
    with np.load(path, allow_pickle=False) as z:
        cfg = json.loads(bytes(z[CONFIG_KEY]).decode())
        spec = ModelSpec.from_dict(cfg["spec"])
        arrays = [np.array(z[n], dtype=np.float32) for n in spec.weight_names()]
        opt = {k[len("__opt__/"):]: np.array(z[k]) for k in z.files if k.startswith("__opt__/")}
    return spec, arrays, cfg, opt


def is_checkpoint(path: str) -> bool:
    if keras_io.is_keras_archive(path) or keras_io.is_hdf5(path):
        return True
    try:
        with np.load(path, allow_pickle=False) as z:
            return CONFIG_KEY in z.files
    except Exception:
        return False
