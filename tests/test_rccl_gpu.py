"""RCCL (backend "nccl") on the GPU box: world-size-1 process groups run the same init, device
binding and device-tensor collectives (all_reduce, all_gather, all_to_all_single, SyncBN sync) the
8-GPU runs use, and bench.py reports the RCCL backend when it owns a process group."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _clean_env(**extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "APNEAUQ_DIST_BACKEND"):
        env.pop(k, None)
    env.update(extra)
    return env


def test_rccl_world1_collectives():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_world1.py")], capture_output=True,
                       text=True, timeout=240, env=_clean_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["pg_backend"] == "nccl" and out["world"] == 1
    for k in ("all_reduce", "all_gather", "all_to_all_members", "all_to_all_single"):
        assert out[k], k
    assert out["syncbn_max_abs_diff"] < 1e-3  # identical statistics up to atomic summation order
    assert out["gather_windows_shape"] == [3, 64]


def test_bench_reports_rccl_world1():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--windows", "512", "--passes",
                        "4", "--steps", "2", "--warmup", "1", "--no-deviation"],
                       capture_output=True, text=True, timeout=240, env=_clean_env(APNEAUQ_FORCE_PG="1"), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["n_gpus"] == 1 and len(out["devices"]) == 1
    assert out["config"]["bn_mode_mcd"] == "batch" and out["dtype"] == "fp32"
    assert out["extra"]["bf16"]["value"] > 0  # the bf16 engine timed in the same run
