"""Keras model-file interop: read and write ``.keras`` (Keras v3 zip) and legacy ``.h5`` models.

The reference saves every model with ``model.save(path.keras)`` (``cnn_baseline_train.py:222-233``,
``train_deep_ensemble_cnns.py:170``) and loads them with ``tf.keras.models.load_model``
(``analyze_mcd_patient_level.py:19,36``, ``analyze_de_patient_level.py:40-58``,
``evaluate_de_global.py:24-38``).  A user switching over brings those files along, so this
module maps them onto :class:`~..models.spec.ModelSpec` + the 38 ``get_weights`` arrays:

* ``.keras`` (TF-Keras >= 2.12 "keras_v3" format): a zip with ``config.json`` (the model's
  ``get_config``), ``metadata.json`` and ``model.weights.h5``, whose layer variables live at
  ``layers/<layer name>/vars/<i>`` in ``trainable + non_trainable`` order (for BN:
  gamma, beta, moving_mean, moving_variance).
* legacy HDF5 (``model.save("x.h5")`` / ``save_weights``): root attribute ``model_config`` (JSON)
  and ``model_weights/<layer>/<weight name>`` datasets listed by the ``weight_names`` attributes.

The architecture is recovered from the config: ``[InputLayer] (Conv1D(relu, same) ->
BatchNormalization -> [MaxPooling1D(2)] -> Dropout) x n -> GlobalAveragePooling1D ->
Dense(1, sigmoid)``, any layer names (the baseline trainer names its layers ``conv1d_1`` ...,
the ensemble trainer leaves Keras' defaults, ``train_deep_ensemble_cnns.py:30-71``).  Other
architectures are rejected with a message naming the offending layer.

Writing produces the same v3 layout, so files this framework trains can be opened by
TF-Keras users, plus one extra member (``apneauq_state.npz``: run metadata and optional Adam
state) that Keras ignores.  HDF5 goes through the pure-Python codec in :mod:`.hdf5` (no h5py in
this image); nothing read from a file is ever executed.
"""
from __future__ import annotations

import datetime
import io
import json
import zipfile
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..models.spec import BlockSpec, ModelSpec
from . import hdf5

KERAS_VERSION = "2.12.0"
STATE_MEMBER = "apneauq_state.npz"


class KerasFormatError(ValueError):
    pass


# ============================================================================ config <-> spec
def _layers_of(config: dict) -> Tuple[str, List[dict]]:
    if config.get("class_name") not in ("Sequential", "Functional", "Model"):
        raise KerasFormatError(f"unsupported model class {config.get('class_name')!r}")
    cfg = config.get("config", {})
    layers = cfg.get("layers", [])
    return cfg.get("name", "model"), layers


def _input_shape(layers: List[dict]) -> Optional[Tuple[int, int]]:
    for ly in layers:
        c = ly.get("config", {})
        for key in ("batch_input_shape", "batch_shape"):
            if key in c and c[key] is not None:
                s = c[key]
                return int(s[-2]), int(s[-1])
        bc = ly.get("build_config", {}).get("input_shape")
        if bc:
            return int(bc[-2]), int(bc[-1])
    return None


def spec_from_config(config: dict) -> Tuple[ModelSpec, str, List[Tuple[str, str]]]:
    """(spec, model name, [(keras layer name, role)]) for a Keras model config.

    ``role`` is ``"conv"``, ``"bn"`` or ``"dense"`` (the layers that own weights), in order.
    """
    name, layers = _layers_of(config)
    shape = _input_shape(layers)
    if shape is None:
        raise KerasFormatError("the config does not record the input shape")
    blocks: List[BlockSpec] = []
    owners: List[Tuple[str, str]] = []
    eps = mom = None
    cur: Optional[dict] = None
    seen_gap = seen_dense = False

    def close():
        nonlocal cur
        if cur is not None:
            if not cur["bn"]:
                raise KerasFormatError(f"Conv1D {cur['name']!r} is not followed by BatchNormalization")
            blocks.append(BlockSpec(cur["filters"], cur["k"], cur["rate"], cur["pool"]))
            cur = None

    for ly in layers:
        cls, c = ly.get("class_name"), ly.get("config", {})
        lname = c.get("name", cls)
        if cls == "InputLayer":
            continue
        if seen_dense:
            raise KerasFormatError(f"layer {lname!r} after the output Dense")
        if cls == "Conv1D":
            close()
            k = c.get("kernel_size")
            k = int(k[0] if isinstance(k, (list, tuple)) else k)
            strides = c.get("strides", [1])
            dil = c.get("dilation_rate", [1])
            if (c.get("padding") != "same" or c.get("activation") != "relu" or not c.get("use_bias", True)
                    or int(np.prod(strides)) != 1 or int(np.prod(dil)) != 1 or int(c.get("groups", 1)) != 1
                    or c.get("data_format", "channels_last") != "channels_last"):
                raise KerasFormatError(f"Conv1D {lname!r}: only padding='same', activation='relu', stride 1, "
                                       "no dilation/groups, channels_last is supported")
            cur = {"name": lname, "filters": int(c["filters"]), "k": k, "bn": False, "pool": False, "rate": 0.0,
                   "stage": "conv"}
            owners.append((lname, "conv"))
        elif cls == "BatchNormalization":
            if cur is None or cur["bn"]:
                raise KerasFormatError(f"BatchNormalization {lname!r} must follow a Conv1D")
            if not (c.get("center", True) and c.get("scale", True)):
                raise KerasFormatError(f"BatchNormalization {lname!r}: center and scale must be on")
            e, m = float(c.get("epsilon", 1e-3)), float(c.get("momentum", 0.99))
            if eps is not None and (e, m) != (eps, mom):
                raise KerasFormatError("BatchNormalization epsilon/momentum differ between blocks")
            eps, mom = e, m
            cur["bn"] = True
            owners.append((lname, "bn"))
        elif cls == "MaxPooling1D":
            ps = c.get("pool_size", [2])
            ps = int(ps[0] if isinstance(ps, (list, tuple)) else ps)
            st = c.get("strides") or [ps]
            st = int(st[0] if isinstance(st, (list, tuple)) else st)
            if cur is None or not cur["bn"] or ps != 2 or st != 2 or c.get("padding", "valid") != "valid":
                raise KerasFormatError(f"MaxPooling1D {lname!r}: only pool_size=2, valid, after BN is supported")
            cur["pool"] = True
        elif cls == "Dropout":
            if cur is None or not cur["bn"]:
                raise KerasFormatError(f"Dropout {lname!r} must follow BatchNormalization")
            cur["rate"] = float(c.get("rate", 0.0))
        elif cls == "GlobalAveragePooling1D":
            close()
            seen_gap = True
        elif cls == "Dense":
            if not seen_gap:
                raise KerasFormatError("Dense before GlobalAveragePooling1D")
            if int(c.get("units", 0)) != 1 or c.get("activation") != "sigmoid" or not c.get("use_bias", True):
                raise KerasFormatError(f"Dense {lname!r}: only Dense(1, sigmoid) is supported")
            owners.append((lname, "dense"))
            seen_dense = True
        else:
            raise KerasFormatError(f"unsupported layer class {cls!r} ({lname!r})")
    if not (seen_gap and seen_dense and blocks):
        raise KerasFormatError("expected Conv1D blocks, GlobalAveragePooling1D and Dense(1, sigmoid)")
    spec = ModelSpec(shape[0], shape[1], tuple(blocks), eps if eps is not None else 1e-3,
                     mom if mom is not None else 0.99)
    return spec, name, owners


def config_from_spec(spec: ModelSpec, name: str = "Alarcon_1D_CNN_Model") -> dict:
    """Keras ``Sequential.get_config()``-shaped config, with the baseline trainer's layer names
    (``cnn_baseline_train.py:59-94``)."""
    L, C = spec.input_length, spec.input_channels

    def layer(cls, cfg, build=None):
        d = {"module": "keras.layers", "class_name": cls, "config": cfg, "registered_name": None}
        if build is not None:
            d["build_config"] = {"input_shape": build}
        return d

    layers = [layer("InputLayer", {"batch_input_shape": [None, L, C], "dtype": "float32", "sparse": False,
                                   "ragged": False, "name": "conv1d_1_input"})]
    ch, ln = spec.channels(), spec.lengths()
    for i, b in enumerate(spec.blocks, 1):
        layers.append(layer("Conv1D", {
            "name": f"conv1d_{i}", "trainable": True, "dtype": "float32", "filters": b.filters,
            "kernel_size": [b.kernel_size], "strides": [1], "padding": "same", "data_format": "channels_last",
            "dilation_rate": [1], "groups": 1, "activation": "relu", "use_bias": True,
            "kernel_initializer": {"module": "keras.initializers", "class_name": "GlorotUniform",
                                   "config": {"seed": None}, "registered_name": None},
            "bias_initializer": {"module": "keras.initializers", "class_name": "Zeros", "config": {},
                                 "registered_name": None},
            "kernel_regularizer": None, "bias_regularizer": None, "activity_regularizer": None,
            "kernel_constraint": None, "bias_constraint": None}, [None, ln[i - 1], ch[i - 1]]))
        layers.append(layer("BatchNormalization", {
            "name": f"batchnorm_{i}", "trainable": True, "dtype": "float32", "axis": [2],
            "momentum": spec.bn_momentum, "epsilon": spec.bn_epsilon, "center": True, "scale": True},
            [None, ln[i - 1], b.filters]))
        if b.pool:
            layers.append(layer("MaxPooling1D", {"name": f"maxpool_{i}", "trainable": True, "dtype": "float32",
                                                 "strides": [2], "pool_size": [2], "padding": "valid",
                                                 "data_format": "channels_last"}))
        layers.append(layer("Dropout", {"name": f"dropout_{i}", "trainable": True, "dtype": "float32",
                                        "rate": b.dropout, "noise_shape": None, "seed": None}))
    layers.append(layer("GlobalAveragePooling1D", {"name": "global_avg_pooling_1d", "trainable": True,
                                                   "dtype": "float32", "data_format": "channels_last",
                                                   "keepdims": False}))
    layers.append(layer("Dense", {"name": "output_layer", "trainable": True, "dtype": "float32", "units": 1,
                                  "activation": "sigmoid", "use_bias": True}, [None, spec.final_channels]))
    return {"module": "keras", "class_name": "Sequential", "config": {"name": name, "layers": layers},
            "registered_name": None, "build_config": {"input_shape": [None, L, C]}}


# ============================================================================ weights
_PER_ROLE = {"conv": 2, "bn": 4, "dense": 2}


def _check_shapes(spec: ModelSpec, arrays: List[np.ndarray]) -> List[np.ndarray]:
    want = spec.weight_shapes()
    if len(arrays) != len(want):
        raise KerasFormatError(f"expected {len(want)} weight arrays, found {len(arrays)}")
    out = []
    for i, (a, s) in enumerate(zip(arrays, want)):
        a = np.asarray(a, dtype=np.float32)
        if tuple(a.shape) != tuple(s):
            raise KerasFormatError(f"weight {spec.weight_names()[i]}: shape {a.shape}, expected {s}")
        out.append(a)
    return out


def _order_to_spec(owners, per_layer: Dict[str, List[np.ndarray]]) -> List[np.ndarray]:
    """Keras layer order (conv, bn, conv, bn, ..., dense) -> get_weights order (the same here)."""
    arrays: List[np.ndarray] = []
    for lname, role in owners:
        vs = per_layer.get(lname)
        if vs is None or len(vs) != _PER_ROLE[role]:
            raise KerasFormatError(f"layer {lname!r}: expected {_PER_ROLE[role]} variables, "
                                   f"found {0 if vs is None else len(vs)}")
        arrays += vs
    return arrays


def _v3_layer_vars(h5: hdf5.File, owners) -> Dict[str, List[np.ndarray]]:
    found: Dict[str, hdf5.Group] = {}
    want = {n for n, _ in owners}
    if "layers" in h5:
        lg = h5["layers"]
        for n in lg.keys():
            if n in want:
                found[n] = lg[n]
    if len(found) < len(want):  # other nestings: any group named like a layer that holds "vars"
        def visit(path, node):
            base = path.rsplit("/", 1)[-1]
            if isinstance(node, hdf5.Group) and base in want and base not in found and "vars" in node:
                found[base] = node
        h5.visit(visit)
    out = {}
    for n, g in found.items():
        vg = g["vars"]
        keys = sorted(vg.keys(), key=lambda k: int(k))
        out[n] = [vg[k].read() for k in keys]
    return out


def _legacy_layer_vars(h5: hdf5.File) -> Dict[str, List[np.ndarray]]:
    root = h5["model_weights"] if "model_weights" in h5 else h5
    out = {}
    names = hdf5.attr_str(root.attrs["layer_names"]) if "layer_names" in root.attrs else root.keys()
    for n in ([names] if isinstance(names, str) else names):
        g = root[n]
        wn = g.attrs.get("weight_names")
        wn = [] if wn is None else hdf5.attr_str(wn)
        out[n] = [g[w].read() for w in ([wn] if isinstance(wn, str) else wn)]
    return out


# ============================================================================ public API
def is_keras_archive(path: str) -> bool:
    try:
        with zipfile.ZipFile(path) as z:
            return "config.json" in z.namelist()
    except (zipfile.BadZipFile, OSError):
        return False


def is_hdf5(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            return f.read(8) == hdf5.SIGNATURE
    except OSError:
        return False


def load(path: str) -> Tuple[ModelSpec, List[np.ndarray], dict, Dict[str, np.ndarray]]:
    """Read a Keras ``.keras`` archive or legacy ``.h5`` model: (spec, 38 arrays, cfg, opt state).

    ``cfg`` has ``name`` (and ``extra`` when the file was written by this framework); ``opt``
    holds the Adam state saved by :func:`save` with ``opt_state`` (empty for Keras-written files:
    their optimizer slots are not imported — the reference only reloads models for inference).
    """
    cfg: dict = {}
    opt: Dict[str, np.ndarray] = {}
    if is_keras_archive(path):
        with zipfile.ZipFile(path) as z:
            config = json.loads(z.read("config.json").decode("utf-8"))
            weights = z.read("model.weights.h5")
            if STATE_MEMBER in z.namelist():
                with np.load(io.BytesIO(z.read(STATE_MEMBER)), allow_pickle=False) as st:
                    cfg = json.loads(bytes(st["__config__"]).decode())
                    opt = {k[len("__opt__/"):]: np.array(st[k]) for k in st.files if k.startswith("__opt__/")}
        spec, name, owners = spec_from_config(config)
        per_layer = _v3_layer_vars(hdf5.File(weights), owners)
    elif is_hdf5(path):
        h5 = hdf5.File(path)
        if "model_config" not in h5.attrs:
            raise KerasFormatError(f"{path}: HDF5 file without a model_config attribute (weights-only files "
                                   "need the architecture; load them with set_weights)")
        config = json.loads(hdf5.attr_str(h5.attrs["model_config"]))
        spec, name, owners = spec_from_config(config)
        per_layer = _legacy_layer_vars(h5)
    else:
        raise KerasFormatError(f"{path}: neither a .keras archive nor an HDF5 model")
    arrays = _check_shapes(spec, _order_to_spec(owners, per_layer))
    cfg.setdefault("name", name)
    cfg.setdefault("format", "keras")
    return spec, arrays, cfg, opt


def _weights_h5(spec: ModelSpec, arrays: List[np.ndarray], opt_iterations: Optional[int] = None) -> bytes:
    w = hdf5.Writer()
    w.create_group("vars")
    names = spec.weight_names()
    groups: Dict[str, List[np.ndarray]] = {}
    for n, a in zip(names, arrays):
        groups.setdefault(n.split("/")[0], []).append(np.asarray(a, dtype=np.float32))
    for lname, vs in groups.items():
        w.create_group(f"layers/{lname}/vars")
        for i, a in enumerate(vs):
            w.create_dataset(f"layers/{lname}/vars/{i}", a)
    for i, b in enumerate(spec.blocks, 1):  # weight-less layers still get (empty) groups, as Keras writes
        w.create_group(f"layers/dropout_{i}/vars")
        if b.pool:
            w.create_group(f"layers/maxpool_{i}/vars")
    w.create_group("layers/global_avg_pooling_1d/vars")
    return w.tobytes()


def save(path: str, spec: ModelSpec, arrays: List[np.ndarray], name: str = "Alarcon_1D_CNN_Model",
         extra: Optional[dict] = None, opt_state: Optional[Dict[str, np.ndarray]] = None) -> str:
    """Write a Keras v3 ``.keras`` archive (config.json, metadata.json, model.weights.h5)."""
    arrays = _check_shapes(spec, list(arrays))
    meta = {"keras_version": KERAS_VERSION, "date_saved": datetime.datetime.now().strftime("%Y-%m-%d@%H:%M:%S")}
    state = {"__config__": np.frombuffer(json.dumps({"spec": spec.to_dict(), "name": name,
                                                     "format": "apneauq-keras-v1",
                                                     "extra": extra or {}}).encode(), dtype=np.uint8)}
    for k, v in (opt_state or {}).items():
        state[f"__opt__/{k}"] = np.asarray(v)
    sbuf = io.BytesIO()
    np.savez(sbuf, **state)
    tmp = path + ".tmp"
    with zipfile.ZipFile(tmp, "w", compression=zipfile.ZIP_STORED) as z:
        z.writestr("metadata.json", json.dumps(meta))
        z.writestr("config.json", json.dumps(config_from_spec(spec, name)))
        z.writestr("model.weights.h5", _weights_h5(spec, arrays))
        z.writestr(STATE_MEMBER, sbuf.getvalue())
    import os

    os.replace(tmp, path)
    return path


def save_legacy_h5(path: str, spec: ModelSpec, arrays: List[np.ndarray], name: str = "Alarcon_1D_CNN_Model") -> str:
    """Write the legacy Keras HDF5 model layout (``model.save("x.h5")``)."""
    arrays = _check_shapes(spec, list(arrays))
    w = hdf5.Writer()
    w.set_attr("/", "keras_version", KERAS_VERSION)
    w.set_attr("/", "backend", "tensorflow")
    w.set_attr("/", "model_config", json.dumps(config_from_spec(spec, name)).encode("utf-8"))
    names = spec.weight_names()
    layer_names: List[str] = []
    per: Dict[str, List[Tuple[str, np.ndarray]]] = {}
    for n, a in zip(names, arrays):
        ln = n.split("/")[0]
        if ln not in per:
            layer_names.append(ln)
            per[ln] = []
        per[ln].append((f"{n}:0", a))
    w.create_group("model_weights")
    w.set_attr("model_weights", "layer_names", [s.encode() for s in layer_names])
    w.set_attr("model_weights", "backend", b"tensorflow")
    w.set_attr("model_weights", "keras_version", KERAS_VERSION.encode())
    for ln in layer_names:
        w.create_group(f"model_weights/{ln}")
        w.set_attr(f"model_weights/{ln}", "weight_names", [wn.encode() for wn, _ in per[ln]])
        for wn, a in per[ln]:
            w.create_dataset(f"model_weights/{ln}/{wn}", np.asarray(a, dtype=np.float32))
    return w.save(path)
