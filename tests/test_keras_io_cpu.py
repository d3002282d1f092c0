"""Keras model-file interop (``utils/keras_io.py``) and the pure-Python HDF5 codec (``utils/hdf5.py``).

The reference saves/loads ``.keras`` files (``cnn_baseline_train.py:230``,
``analyze_mcd_patient_level.py:36``).  Neither TensorFlow nor h5py is installed here and the
reference ships no model file, so files written by libhdf5 cannot be read in these tests:
parity with Keras-written files is *unpinned*.  What is pinned: round trips through our writer,
a hand-assembled "new-style" HDF5 file (v2 superblock, v2 object headers, link messages, compact
layout) exercising the reader paths our writer never emits, the Keras config -> spec mapping for
both layer-naming schemes the reference uses, and rejection of unsupported architectures.
"""
import json
import struct
import zipfile

import numpy as np
import pytest

from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC, BlockSpec, ModelSpec
from uncertaintyquantification_sleepapnea_1dcnn_amd.utils import hdf5, keras_io
from uncertaintyquantification_sleepapnea_1dcnn_amd.utils.checkpoint import load_weights, save_weights


def _rand_arrays(spec, seed=0):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(s).astype(np.float32) for s in spec.weight_shapes()]


def test_hdf5_roundtrip_types_and_attrs():
    w = hdf5.Writer()
    data = {
        "a/b/f32": np.arange(24, dtype=np.float32).reshape(2, 3, 4),
        "a/f64": np.linspace(0, 1, 7),
        "a/i64": np.array(-5, dtype=np.int64),
        "u8": np.arange(10, dtype=np.uint8),
        "s": np.array([b"ab", b"cde"]),
    }
    for k, v in data.items():
        w.create_dataset(k, v)
    w.create_group("empty")
    w.set_attr("/", "vlen", "héllo wörld")
    w.set_attr("/", "fixed", b"xyz")
    w.set_attr("a", "names", [b"n1", b"name2"])
    w.set_attr("a/f64", "scale", np.array([1.5, 2.5], dtype=np.float32))
    f = hdf5.File(w.tobytes())
    assert sorted(f.keys()) == ["a", "empty", "s", "u8"]
    assert f["empty"].keys() == []
    for k, v in data.items():
        got = f[k].read()
        assert got.shape == v.shape and got.dtype == v.dtype.newbyteorder("<")
        np.testing.assert_array_equal(got, v)
    assert hdf5.attr_str(f.attrs["vlen"]) == "héllo wörld"
    assert hdf5.attr_str(f.attrs["fixed"]) == "xyz"
    assert hdf5.attr_str(f["a"].attrs["names"]) == ["n1", "name2"]
    np.testing.assert_array_equal(f["a/f64"].attrs["scale"], [1.5, 2.5])
    with pytest.raises(KeyError):
        f["a/missing"]


def test_hdf5_superblock_layout():
    """Byte-level spot checks of the v0 superblock the writer emits (HDF5 spec, section II.A)."""
    b = hdf5.Writer().tobytes()
    assert b[:8] == hdf5.SIGNATURE
    assert b[8] == 0 and b[13] == 8 and b[14] == 8  # version 0, 8-byte offsets and lengths
    eof = struct.unpack_from("<Q", b, 40)[0]
    assert eof == len(b)
    assert struct.unpack_from("<I", b, 72)[0] == 1  # root entry caches the symbol table (type 1)


def _new_style_file() -> bytes:
    """v2 superblock -> OHDR root group with one link message -> OHDR dataset (compact layout)."""
    arr = np.arange(6, dtype=np.float32).reshape(2, 3)
    dt = bytes([0x11, 0x20, 0x1F, 0]) + struct.pack("<I", 4) + struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
    sp = struct.pack("<BBBB", 2, 2, 0, 1) + struct.pack("<QQ", 2, 3)
    lay = struct.pack("<BBH", 3, 0, arr.nbytes) + arr.tobytes()

    def ohdr(msgs):
        body = b"".join(struct.pack("<BHB", t, len(d), 0) + d for t, d in msgs)
        return b"OHDR" + bytes([2, 0x02]) + struct.pack("<I", len(body)) + body + b"\0\0\0\0"

    ds = ohdr([(0x01, sp), (0x03, dt), (0x08, lay)])
    sb_len = 8 + 4 + 4 * 8 + 4
    ds_addr = sb_len
    name = b"weights"
    link = bytes([1, 0x00, len(name)]) + name + struct.pack("<Q", ds_addr)
    linfo = bytes([0, 0]) + struct.pack("<QQ", hdf5.UNDEF, hdf5.UNDEF)
    root = ohdr([(0x02, linfo), (0x06, link)])
    root_addr = ds_addr + len(ds)
    eof = root_addr + len(root)
    sb = hdf5.SIGNATURE + bytes([2, 8, 8, 0]) + struct.pack("<QQQQ", 0, hdf5.UNDEF, eof, root_addr) + b"\0\0\0\0"
    assert len(sb) == sb_len
    return sb + ds + root


def test_hdf5_reader_new_style_groups_and_compact_layout():
    f = hdf5.File(_new_style_file())
    assert f.keys() == ["weights"]
    np.testing.assert_array_equal(f["weights"].read(), np.arange(6, dtype=np.float32).reshape(2, 3))


@pytest.mark.parametrize("pool", [False, True])
def test_keras_archive_roundtrip(tmp_path, pool):
    spec = ModelSpec.with_input((60, 4), pool=pool)
    arrays = _rand_arrays(spec, 1)
    p = str(tmp_path / "m.keras")
    save_weights(p, spec, arrays, "Alarcon_1D_CNN_Model", extra={"seed": 7},
                 opt_state={"iterations": np.array(3)})
    with zipfile.ZipFile(p) as z:
        names = set(z.namelist())
        assert {"config.json", "metadata.json", "model.weights.h5"} <= names
        cfg = json.loads(z.read("config.json"))
        h5 = hdf5.File(z.read("model.weights.h5"))
    assert cfg["class_name"] == "Sequential"
    classes = [ly["class_name"] for ly in cfg["config"]["layers"]]
    assert classes.count("Conv1D") == 6 and classes.count("MaxPooling1D") == (6 if pool else 0)
    np.testing.assert_array_equal(h5["layers/batchnorm_3/vars/3"].read(), arrays[6 * 2 + 5])  # moving_variance
    spec2, arrays2, cfg2, opt = load_weights(p)
    assert spec2 == spec
    assert cfg2["extra"]["seed"] == 7 and int(opt["iterations"]) == 3
    for a, b in zip(arrays, arrays2):
        np.testing.assert_array_equal(a, b)


def test_keras_archive_without_state_member(tmp_path):
    """A Keras-written archive has no apneauq member: spec and weights come from config + h5 alone."""
    arrays = _rand_arrays(DEFAULT_SPEC, 2)
    src = str(tmp_path / "a.keras")
    keras_io.save(src, DEFAULT_SPEC, arrays)
    dst = str(tmp_path / "b.keras")
    with zipfile.ZipFile(src) as zi, zipfile.ZipFile(dst, "w") as zo:
        for n in zi.namelist():
            if n != keras_io.STATE_MEMBER:
                zo.writestr(n, zi.read(n))
    spec, arrays2, cfg, opt = load_weights(dst)
    assert spec == DEFAULT_SPEC and cfg["name"] == "Alarcon_1D_CNN_Model" and opt == {}
    for a, b in zip(arrays, arrays2):
        np.testing.assert_array_equal(a, b)


def test_ensemble_trainer_default_layer_names(tmp_path):
    """``train_deep_ensemble_cnns.py:30-71`` leaves layer names to Keras (conv1d, batch_normalization,
    conv1d_1, ...): the importer keys on the config, not on names."""
    arrays = _rand_arrays(DEFAULT_SPEC, 3)
    cfg = keras_io.config_from_spec(DEFAULT_SPEC)
    counters = {}
    rename = {}
    for ly in cfg["config"]["layers"]:
        base = {"Conv1D": "conv1d", "BatchNormalization": "batch_normalization", "Dropout": "dropout",
                "GlobalAveragePooling1D": "global_average_pooling1d", "Dense": "dense",
                "InputLayer": "input_1"}[ly["class_name"]]
        k = counters.get(base, 0)
        counters[base] = k + 1
        new = base if k == 0 else f"{base}_{k}"
        rename[ly["config"]["name"]] = new
        ly["config"]["name"] = new
    w = hdf5.Writer()
    owners = [n.split("/")[0] for n in DEFAULT_SPEC.weight_names()]
    idx = {}
    for n, a in zip(owners, arrays):
        i = idx.get(n, 0)
        idx[n] = i + 1
        w.create_dataset(f"layers/{rename[n]}/vars/{i}", a)
    p = str(tmp_path / "AlCNN_smote_seed21.keras")
    with zipfile.ZipFile(p, "w") as z:
        z.writestr("config.json", json.dumps(cfg))
        z.writestr("metadata.json", "{}")
        z.writestr("model.weights.h5", w.tobytes())
    spec, arrays2, _, _ = load_weights(p)
    assert spec == DEFAULT_SPEC
    for a, b in zip(arrays, arrays2):
        np.testing.assert_array_equal(a, b)


def test_legacy_h5_roundtrip(tmp_path):
    spec = ModelSpec(30, 1, tuple(BlockSpec(f, k, r) for f, k, r in [(16, 5, 0.1), (8, 3, 0.2)]))
    arrays = _rand_arrays(spec, 4)
    p = str(tmp_path / "m.h5")
    save_weights(p, spec, arrays, "tiny")
    f = hdf5.File(p)
    assert hdf5.attr_str(f["model_weights"].attrs["layer_names"])[0] == "conv1d_1"
    assert f["model_weights/conv1d_1/conv1d_1/kernel:0"].shape == (5, 1, 16)
    spec2, arrays2, cfg, _ = load_weights(p)
    assert spec2 == spec and cfg["name"] == "tiny"
    for a, b in zip(arrays, arrays2):
        np.testing.assert_array_equal(a, b)


def test_load_model_predictions_match(tmp_path):
    import torch

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D, load_model

    m = AlarconCNN1D(seed=5, device="cpu")
    p = m.save(str(tmp_path / "alarcon_cnn_model.keras"))
    m2 = load_model(p, device="cpu")
    x = torch.randn(16, 60, 4)
    np.testing.assert_array_equal(m.predict(x), m2.predict(x))


@pytest.mark.parametrize("mutate,msg", [
    (lambda c: c["config"]["layers"][1]["config"].update(padding="valid"), "padding='same'"),
    (lambda c: c["config"]["layers"][-1]["config"].update(units=2), "Dense"),
    (lambda c: c["config"]["layers"].insert(3, {"class_name": "LSTM", "config": {"name": "lstm"}}), "LSTM"),
    (lambda c: c["config"]["layers"].pop(2), "BatchNormalization"),
])
def test_unsupported_architectures_rejected(mutate, msg):
    cfg = keras_io.config_from_spec(DEFAULT_SPEC)
    mutate(cfg)
    with pytest.raises(keras_io.KerasFormatError, match=msg):
        keras_io.spec_from_config(cfg)
