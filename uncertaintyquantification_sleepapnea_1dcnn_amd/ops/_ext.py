"""Loader for the in-tree HIP extension (``_apneauq_hip.so``, built by ``csrc/build.py``).

The extension registers ``torch.ops.apneauq.*``.  On a machine with a GPU the framework refuses
to silently fall back to eager PyTorch for an op that has a HIP kernel: :func:`require` raises
with the build command instead.  Set ``APNEAUQ_ALLOW_FALLBACK=1`` to permit the eager reference
path (used only by the CPU-only test tier).
"""
from __future__ import annotations

import os
import threading

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# APNEAUQ_SO_PATH loads a probe variant built with csrc/build.py APNEAUQ_SO_OUT=... (timing ablations only)
SO_PATH = os.environ.get("APNEAUQ_SO_PATH") or os.path.join(_PKG, "_apneauq_hip.so")
_lock = threading.Lock()
_state = {"loaded": False, "error": None}


def load(build_if_missing: bool = False) -> bool:
    """Load the extension once; returns True on success."""
    with _lock:
        if _state["loaded"]:
            return True
        if not os.path.exists(SO_PATH) and build_if_missing:
            from ..csrc import build as _build

            _build.build()
        if not os.path.exists(SO_PATH):
            _state["error"] = f"{SO_PATH} not built"
            return False
        try:
            torch.ops.load_library(SO_PATH)
            _state["loaded"] = True
            return True
        except Exception as e:  # pragma: no cover - depends on the box
            _state["error"] = repr(e)
            return False


def available() -> bool:
    return load()


def gpu_available() -> bool:
    return torch.cuda.is_available()


def fallback_allowed() -> bool:
    return os.environ.get("APNEAUQ_ALLOW_FALLBACK", "0") == "1" or not torch.cuda.is_available()


def require() -> None:
    """Raise loudly if the HIP extension cannot be used on this (GPU) machine."""
    if not load():
        raise RuntimeError(
            "apneauq HIP extension is not available "
            f"({_state['error']}); build it with "
            "`python -m uncertaintyquantification_sleepapnea_1dcnn_amd.csrc.build`")


def ops():
    require()
    return torch.ops.apneauq
