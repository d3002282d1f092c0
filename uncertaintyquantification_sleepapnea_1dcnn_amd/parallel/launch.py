"""Self-launch of one worker process per GPU (``python bench.py --gpus N`` without torchrun).

The reference has no launcher at all (single process); the MI355X framework runs one
process per GPU over RCCL.  ``torchrun`` sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; when a
script is started directly with ``--gpus N > 1`` this module plays torchrun's role:

* the parent spawns N fresh interpreters of the same script (``subprocess``, never ``exec``) with
  the rendezvous environment (127.0.0.1, a free port), **before anything touches the GPU** — this
  module does not import torch, and callers invoke it before their own torch import;
* every worker binds ``cuda:LOCAL_RANK`` and checks ``WORLD_SIZE == --gpus`` (``check_world``);
* the first worker failure terminates the others; the parent exits with the first non-zero code.

Only rank 0's stdout is meaningful (the workers inherit the parent's stdout / stderr).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence

ENV_FLAG = "APNEAUQ_LAUNCHED"


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def under_launcher() -> bool:
    """True inside torchrun or a worker spawned by :func:`maybe_spawn`."""
    return "WORLD_SIZE" in os.environ


def worker_env(rank: int, world: int, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                ENV_FLAG: "1"})
    # dmabuf IPC is the only mode the host driver supports (RCCL / tensor sharing across processes)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn(n: int, cmd: Sequence[str], poll_s: float = 0.2) -> int:
    """Run ``cmd`` as ``n`` ranks on 127.0.0.1; returns 0 or the first failing rank's exit code."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(n):
        procs.append(subprocess.Popen(list(cmd), env=worker_env(r, n, port), start_new_session=False))
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                code = p.poll()
                if code is None:
                    alive += 1
                elif code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
            if rc != 0 or alive == 0:
                break
            time.sleep(poll_s)
    finally:
        if rc != 0:
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGTERM)
            deadline = time.time() + 20
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
        else:
            for p in procs:
                p.wait()
    return rc


def maybe_spawn(n_gpus: int, script: str, argv: Sequence[str]) -> Optional[int]:
    """Spawn ``n_gpus`` workers of ``script`` when not already under a launcher.

    Returns None when the caller should simply run (one process, or already a worker / under
    torchrun), else the exit code the parent should exit with.
    """
    if under_launcher() or n_gpus <= 1:
        return None
    return spawn(n_gpus, [sys.executable, os.path.abspath(script), *argv])


def check_world(expected: int, world: int, device_count: Optional[int] = None, device_type: str = "cuda") -> None:
    """Refuse to measure on the wrong number of ranks / GPUs (exit code 3)."""
    if world != expected:
        sys.stderr.write(f"apneauq: --gpus {expected} but WORLD_SIZE={world}; refusing to run\n")
        raise SystemExit(3)
    if device_type == "cuda" and device_count is not None and device_count < world:
        if os.environ.get("APNEAUQ_REHEARSE_SHARED_GPU") == "1":  # multi-rank rehearsal on one card (gloo)
            sys.stderr.write(f"apneauq: REHEARSAL: {world} ranks share {device_count} GPU(s); not a measurement\n")
            return
        sys.stderr.write(f"apneauq: {world} ranks but only {device_count} visible GPU(s); refusing to share devices\n")
        raise SystemExit(3)
