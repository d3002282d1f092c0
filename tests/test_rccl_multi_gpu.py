"""Multi-rank RCCL (backend "nccl", one process per GPU over xGMI) on boxes with >= 2 GPUs.

Skipped on a 1-GPU box (RCCL cannot host two ranks on one device; tests/test_rccl_gpu.py covers world
size 1 there).  Self-launches 2 and N = device_count() ranks with parallel.launch.spawn and checks,
against the same computation on one rank (tests/rccl_multi_worker.py):
  * batch-BN MC Dropout with SyncBN over the window shards: probabilities within 1e-6, moving
    statistics within 1e-6 (the reference's model(x, training=True) loop, uq_techniques.py:22);
  * Deep-Ensemble member-parallel inference + all_to_all: bitwise equal (uq_techniques.py:29);
  * deterministic data-parallel training step: gradient within 1e-7 x scale, all ranks bitwise equal;
  * bench.py --gpus N: n_gpus == N, backend nccl, N distinct devices."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NGPU = torch.cuda.device_count() if torch.cuda.is_available() else 0
WORLDS = sorted({2, NGPU}) if NGPU >= 2 else [2]


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "APNEAUQ_DIST_BACKEND",
              "APNEAUQ_REHEARSE_SHARED_GPU"):
        env.pop(k, None)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    return env


def _run_worker(world, tmp_path, **extra):
    res = tmp_path / "r.json"
    env = _env()
    env["APNEAUQ_RESULT"] = str(res)
    env.update(extra)
    code = ("import sys; sys.path.insert(0, %r); from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import "
            "launch; sys.exit(launch.spawn(%d, [sys.executable, %r]))" % (ROOT, world, os.path.join(ROOT, "tests",
                                                                                                    "rccl_multi_worker.py")))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(res.read_text())


def _check(out):
    assert out["mcd_max_abs_dp"] <= 1e-6, out
    assert out["mcd_moving_stats_max_abs"] <= 1e-6, out
    assert out["de_bitwise"], out
    assert out["dp_grad_max_abs"] <= 1e-6 and out["dp_stats_max_abs"] <= 1e-6, out
    assert out["dp_ranks_bitwise_equal"], out


@pytest.mark.skipif(NGPU < 2, reason="needs >= 2 GPUs for multi-rank RCCL")
@pytest.mark.parametrize("world", WORLDS)
def test_rccl_multi_rank_matches_one_rank(world, tmp_path):
    out = _run_worker(world, tmp_path)
    assert out["world"] == world and out["backend"] == "nccl"
    assert len(set(out["devices"])) == world
    _check(out)


@pytest.mark.skipif(NGPU != 1, reason="rehearsal of the multi-rank worker for one-GPU boxes")
def test_multi_rank_worker_rehearsal_on_one_gpu(tmp_path):
    """The same worker with 2 ranks sharing the one GPU over gloo (RCCL refuses two ranks per device):
    validates the sharded / member-parallel / DP logic the multi-GPU test runs; not an RCCL test."""
    out = _run_worker(2, tmp_path, APNEAUQ_DIST_BACKEND="gloo", APNEAUQ_REHEARSE_SHARED_GPU="1")
    assert out["world"] == 2 and out["backend"] == "gloo"
    _check(out)


@pytest.mark.skipif(NGPU < 2, reason="needs >= 2 GPUs for multi-rank RCCL")
def test_bench_multi_gpu_reports_rccl():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(NGPU), "--windows", "512",
                        "--passes", "4", "--members", "8" if 8 % NGPU == 0 else str(NGPU), "--steps", "2", "--warmup",
                        "1", "--no-deviation", "--no-secondary"],
                       capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == NGPU and out["backend"] == "nccl"
    assert len(set(out["devices"])) == NGPU
    assert out["dtype"] == "fp32" and out["value"] > 0
