"""Tracing / profiling hooks (SURVEY §5 "Tracing / profiling").

The reference only brackets MCD, DE and the bootstrap with ``time.time()`` prints
(``uq_techniques.py:21-23,28-31,339,347``).  Here:

* :class:`Timer` — a region timer that uses HIP events on a GPU stream (device time, no host
  sync inside the region) and ``perf_counter`` on CPU; results accumulate in :data:`TIMINGS`
  and are optionally streamed to the JSONL metrics sink;
* :func:`region` — ``torch.profiler.record_function`` + :class:`Timer` in one context manager, so
  regions show up by name in a ``torch.profiler`` / ``rocprofv3 --marker-trace`` timeline;
* :func:`profile` — run a block under ``torch.profiler`` (CPU + HIP activities) and export a
  Chrome trace and a kernel table;
* per-kernel device counters come from ``rocprofv3`` (``tools/prof_summary.py`` turns its
  ``--stats`` CSV into the tables under ``profiles/``).
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch

from .logging import log_metrics

TIMINGS: Dict[str, List[float]] = defaultdict(list)


class Timer:
    """``with Timer("mcd") as t: ...``; ``t.ms`` after exit (synchronises the event only)."""

    def __init__(self, name: str, device: Optional[torch.device] = None, stream_to_jsonl: bool = False):
        self.name = name
        self.cuda = (device is None and torch.cuda.is_available()) or (device is not None and torch.device(device).type == "cuda")
        self.stream_to_jsonl = stream_to_jsonl
        self.ms: Optional[float] = None

    def __enter__(self):
        if self.cuda:
            self._e0 = torch.cuda.Event(enable_timing=True)
            self._e1 = torch.cuda.Event(enable_timing=True)
            self._e0.record()
        else:
            self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.cuda:
            self._e1.record()
            self._e1.synchronize()
            self.ms = self._e0.elapsed_time(self._e1)
        else:
            self.ms = (time.perf_counter() - self._t0) * 1e3
        TIMINGS[self.name].append(self.ms)
        if self.stream_to_jsonl:
            log_metrics({"event": "timing", "region": self.name, "ms": self.ms})
        return False


@contextlib.contextmanager
def region(name: str, timed: bool = False):
    """Named region for profilers; ``timed=True`` also measures it with :class:`Timer`."""
    with torch.profiler.record_function(name):
        if timed:
            with Timer(name) as t:
                yield t
        else:
            yield None


def summary() -> Dict[str, Dict[str, float]]:
    out = {}
    for k, v in TIMINGS.items():
        out[k] = {"n": len(v), "total_ms": sum(v), "mean_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v)}
    return out


def reset() -> None:
    TIMINGS.clear()


@contextlib.contextmanager
def profile(out_dir: str = "gpurun_out/torch_profile", row_limit: int = 30, sort_by: Optional[str] = None):
    """Profile the enclosed block; writes ``trace.json`` (Chrome/Perfetto) and ``kernels.txt``."""
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    os.makedirs(out_dir, exist_ok=True)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    prof.export_chrome_trace(os.path.join(out_dir, "trace.json"))
    key = sort_by or ("self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total")
    with open(os.path.join(out_dir, "kernels.txt"), "w") as f:
        f.write(prof.key_averages().table(sort_by=key, row_limit=row_limit))
