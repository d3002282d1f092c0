"""Collective accounting: how many collectives a step issues, how many bytes they move and how long
they occupy the compute stream, per phase.

The reference has no collectives at all: every one here replaces a serial loop of
``uq_techniques.py:22,29`` or a single-device reduction.  A multi-GPU run that scales sub-linearly
must be attributable from its own record, so ``bench.py`` meters a few steps after its timed region
and reports ``extra.comm``:

    {"steps": k, "phases": {phase: {op: {"count", "bytes", "ms"}}}}   (per step)

Usage::

    m = comm.CommMeter()
    with comm.metering(m):
        m.phase("mcd"); ...            # call sites go through comm.run(...)
    m.summary()

``run(op, tensors, fn)`` executes ``fn()`` (the collective) and, when a meter is active, counts it,
adds the bytes of ``tensors`` and brackets it with HIP events on the current stream (CUDA tensors) or
a host clock (gloo / CPU).  Without an active meter it is a plain call.
"""
from __future__ import annotations

import contextlib
import time
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Union

import torch


class CommMeter:
    def __init__(self):
        self._phase = "default"
        self.steps = 0
        self._rec: Dict[str, Dict[str, List]] = {}  # phase -> op -> [count, bytes, host_ms, [event pairs]]

    def phase(self, name: str) -> None:
        self._phase = name

    def step(self) -> None:
        self.steps += 1

    def _slot(self, op: str) -> List:
        return self._rec.setdefault(self._phase, {}).setdefault(op, [0, 0, 0.0, []])

    def record(self, op: str, nbytes: int, fn: Callable, device: Optional[torch.device]):
        s = self._slot(op)
        s[0] += 1
        s[1] += int(nbytes)
        if device is not None and device.type == "cuda":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn()
            e1.record()
            s[3].append((e0, e1))
            return out
        t0 = time.perf_counter()
        out = fn()
        s[2] += (time.perf_counter() - t0) * 1e3
        return out

    def summary(self) -> Dict:
        """Per-step averages (synchronises the device to read the events)."""
        if any(s[3] for ops in self._rec.values() for s in ops.values()) and torch.cuda.is_available():
            torch.cuda.synchronize()
        k = max(self.steps, 1)
        phases = {}
        for ph, ops in self._rec.items():
            phases[ph] = {}
            for op, (cnt, nb, host_ms, evs) in ops.items():
                ms = host_ms + sum(a.elapsed_time(b) for a, b in evs)
                phases[ph][op] = {"count": round(cnt / k, 3), "bytes": round(nb / k, 1), "ms": round(ms / k, 4)}
        return {"steps": self.steps, "phases": phases}


_ACTIVE: Optional[CommMeter] = None


def active() -> Optional[CommMeter]:
    return _ACTIVE


@contextlib.contextmanager
def metering(m: CommMeter):
    global _ACTIVE
    old, _ACTIVE = _ACTIVE, m
    try:
        yield m
    finally:
        _ACTIVE = old


def run(op: str, tensors: Union[torch.Tensor, Sequence[torch.Tensor]], fn: Callable):
    """Execute the collective ``fn()``; account it under ``op`` when a meter is active."""
    m = _ACTIVE
    if m is None:
        return fn()
    ts: Iterable[torch.Tensor] = [tensors] if isinstance(tensors, torch.Tensor) else tensors
    ts = list(ts)
    nbytes = sum(t.numel() * t.element_size() for t in ts)
    return m.record(op, nbytes, fn, ts[0].device if ts else None)
