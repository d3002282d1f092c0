"""bench.py driver contract on the CPU: ``--gpus N`` self-launches N ranks (gloo dry run) and the
reported ``n_gpus`` / backend / devices / aggregates match; the UQ aggregates do not depend on the
rank count (masks keyed by global window index, SyncBN over the whole window set)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", *args],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_bench_self_launch_two_ranks_matches_one():
    common = ["--passes", "3", "--members", "2", "--steps", "1", "--warmup", "1", "--no-secondary"]
    two = _bench("--gpus", "2", "--windows", "24", *common)
    one = _bench("--gpus", "1", "--windows", "48", *common)
    assert two["n_gpus"] == 2 and two["backend"] == "gloo" and len(two["devices"]) == 2
    assert one["n_gpus"] == 1
    assert two["config"]["global_batch"] == one["config"]["global_batch"] == 48
    for k in ("mcd_mean_entropy", "de_mean_mutual_info"):
        assert abs(two["extra"][k] - one["extra"][k]) < 1e-5, (k, two["extra"][k], one["extra"][k])
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling", "dtype",
              "data", "config"):
        assert k in two


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                        "--windows", "8", "--passes", "1", "--members", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr


@pytest.mark.parametrize("n", [1, 3])
def test_launch_spawn_exit_codes(n, tmp_path):
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel import launch

    script = tmp_path / "w.py"
    script.write_text("import os, sys\nr = int(os.environ['RANK'])\n"
                      "assert os.environ['WORLD_SIZE'] == '%d' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "sys.exit(7 if r == %d - 1 and %d > 1 else 0)\n" % (n, n, n))
    rc = launch.spawn(n, [sys.executable, str(script)])
    assert rc == (7 if n > 1 else 0)


def test_bench_comm_block_counts_collectives():
    """extra.comm: the metered steps after the timed region report, per step and phase,
    how many collectives ran and their bytes.  2 ranks, T=3 passes, M=2 members (member-parallel):
    MC Dropout = one SyncBN all-reduce of (sum, sum of squares) per BN layer and pass, plus one of the
    row count (6 layers x 2 x T); Deep Ensemble = one all_to_all of the member probabilities; then one
    all-reduce of the 2 x 9 fp64 aggregate sums."""
    out = _bench("--gpus", "2", "--windows", "24", "--passes", "3", "--members", "2", "--steps", "1", "--warmup", "1",
                 "--no-secondary", "--comm-steps", "2")
    c = out["extra"]["comm"]
    assert c["steps"] == 2
    ph = c["phases"]
    chans = 128 + 192 + 224 + 96 + 256 + 96
    assert ph["mcd"]["syncbn_all_reduce"]["count"] == 6 * 2 * 3
    assert ph["mcd"]["syncbn_all_reduce"]["bytes"] == 3 * (chans * 2 * 8 + 6 * 8)
    assert ph["de"]["all_to_all"]["count"] == 1
    assert ph["de"]["all_to_all"]["bytes"] == 2 * 1 * 24 * 4  # (ranks, members per rank, windows per rank) fp32
    assert ph["aggregate"]["all_reduce"]["count"] == 1 and ph["aggregate"]["all_reduce"]["bytes"] == 2 * 9 * 8
    for p in ph.values():
        for v in p.values():
            assert v["ms"] >= 0.0
