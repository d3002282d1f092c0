"""Auxiliary subsystems: config, JSONL metrics, tracing, fault injection + recovery."""
import json
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from uncertaintyquantification_sleepapnea_1dcnn_amd.utils import faults, tracing
from uncertaintyquantification_sleepapnea_1dcnn_amd.utils.config import RunConfig
from uncertaintyquantification_sleepapnea_1dcnn_amd.utils.logging import JsonlWriter, get_logger

from .dist_utils import run_ranks


def test_config_layers(tmp_path, monkeypatch):
    c = RunConfig()
    assert c.mcd_passes == 50 and c.n_bootstrap == 100 and c.seed == 2025 and c.bn_mode == "batch"
    p = tmp_path / "c.yaml"
    p.write_text("mcd_passes: 20\nbn_mode: running\n")
    monkeypatch.setenv("APNEAUQ_SEED", "7")
    monkeypatch.setenv("APNEAUQ_POOL", "true")
    c = RunConfig.load(str(p), de_members=8)
    assert (c.mcd_passes, c.bn_mode, c.seed, c.pool, c.de_members) == (20, "running", 7, True, 8)
    assert RunConfig.from_dict(json.loads(c.to_json())) == c
    assert all(b.pool for b in c.spec().blocks)
    with pytest.raises(ValueError):
        RunConfig(bn_mode="train")
    with pytest.raises(KeyError):
        RunConfig.from_dict({"nope": 1})


def test_jsonl_and_logger(tmp_path):
    w = JsonlWriter(str(tmp_path / "m.jsonl"))
    w.write({"a": np.float32(1.5), "b": torch.tensor(2.0), "c": float("nan")}, step=3)
    w.write({"arr": np.arange(3)})
    rec = JsonlWriter.read(str(tmp_path / "m.jsonl"))
    assert rec[0]["a"] == 1.5 and rec[0]["b"] == 2.0 and rec[0]["c"] == "nan" and rec[0]["step"] == 3
    assert rec[1]["arr"] == [0, 1, 2] and rec[0]["rank"] == 0
    get_logger("apneauq.test").info("hello")


def test_tracing_timer_and_profile(tmp_path):
    tracing.reset()
    with tracing.region("work", timed=True) as t:
        torch.randn(64, 64) @ torch.randn(64, 64)
    assert t.ms is not None and tracing.summary()["work"]["n"] == 1
    with tracing.profile(str(tmp_path / "prof")):
        torch.randn(32, 32).sum()
    assert os.path.exists(tmp_path / "prof" / "trace.json") and os.path.exists(tmp_path / "prof" / "kernels.txt")


def test_fault_spec_matching(monkeypatch):
    monkeypatch.setenv("APNEAUQ_FAULT", "ensemble.before_save:member=2|fit.epoch_end:epoch=1;rank=0")
    assert faults.armed("ensemble.before_save", member=2)
    assert not faults.armed("ensemble.before_save", member=1)
    assert faults.armed("fit.epoch_end", epoch=1)
    monkeypatch.setenv("RANK", "1")
    assert not faults.armed("fit.epoch_end", epoch=1)


# ------------------------------------------------------------- epoch-level fault tolerance
def _fit_child(backup_dir, out, fault):
    if fault:
        os.environ["APNEAUQ_FAULT"] = fault
    torch.set_num_threads(2)
    from uncertaintyquantification_sleepapnea_1dcnn_amd.data.synthetic import synthetic_windows
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.training.callbacks import BackupAndRestore, JsonlLogger

    x, y, _ = synthetic_windows(128, seed=4)
    m = AlarconCNN1D(seed=11, device="cpu")
    cbs = [JsonlLogger(os.path.join(os.path.dirname(out), "log.jsonl"))]
    if backup_dir:
        cbs.append(BackupAndRestore(backup_dir))
    m.fit(x, y.astype(np.float32), epochs=3, batch_size=32, callbacks=cbs, verbose=0)
    np.savez(out, *m.get_weights())


def _spawn(*args):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_fit_child, args=args)
    p.start()
    p.join(300)
    return p.exitcode


def test_backup_and_restore_resumes_bitwise(tmp_path):
    ref, res = str(tmp_path / "ref.npz"), str(tmp_path / "res.npz")
    assert _spawn(None, ref, None) == 0
    bd = str(tmp_path / "bk")
    assert _spawn(bd, res, "fit.epoch_end:epoch=1") == 17  # killed after epoch index 1
    assert os.path.exists(os.path.join(bd, "backup.npz")) and not os.path.exists(res)
    assert _spawn(bd, res, None) == 0  # resumes at epoch index 2
    assert not os.path.exists(os.path.join(bd, "backup.npz"))
    a, b = np.load(ref), np.load(res)
    for k in a.files:
        np.testing.assert_array_equal(a[k], b[k])
    epochs = [r["epoch"] for r in JsonlWriter.read(str(tmp_path / "log.jsonl")) if r["event"] == "epoch"]
    assert epochs == [0, 1, 2, 0, 1, 2]  # ref run, then the killed run (0, 1), then the resumed run (2)


# ------------------------------------------------------------- member-level fault tolerance
def _ens_fault(rank, world, save_dir, fault):
    if fault:
        os.environ["APNEAUQ_FAULT"] = fault
    from uncertaintyquantification_sleepapnea_1dcnn_amd.data.synthetic import synthetic_windows
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel.ensemble import train_ensemble

    x, y, _ = synthetic_windows(96, seed=2)
    return train_ensemble(x, y.astype(np.float32), num_models=3, seed_base=7, save_dir=save_dir, epochs=1,
                          batch_size=32, verbose=0, device="cpu")


def test_ensemble_killed_rank_resume(tmp_path):
    d = str(tmp_path / "ens")
    with pytest.raises(Exception):
        run_ranks(_ens_fault, 2, (d, "ensemble.before_save:member=2"))  # rank 0 dies before saving member 2
    names = sorted(os.listdir(d)) if os.path.isdir(d) else []
    survived = {n: os.path.getmtime(os.path.join(d, n)) for n in names if n.startswith("AlCNN")}
    assert "AlCNN_smote_seed21.keras" in survived and "AlCNN_smote_seed23.keras" not in survived
    paths = run_ranks(_ens_fault, 2, (d, None))[0]
    assert all(os.path.exists(p) for p in paths)
    for n, t in survived.items():
        assert os.path.getmtime(os.path.join(d, n)) == t  # finished members are not retrained
    assert not [n for n in os.listdir(d) if n.startswith(".backup")]  # backups cleaned up
