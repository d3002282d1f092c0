"""Logging and the JSONL metrics stream (SURVEY §5 "Metrics / logging / observability").

The reference only ``print``s (Keras ``verbose=2`` epoch lines, wall-clock prints in
``uq_techniques.py:23,31,347``) and never persists its ``History``.  Here:

* :func:`get_logger` — a ``logging`` logger whose records carry the distributed rank;
* :class:`JsonlWriter` — append-only JSON-lines sink (one object per line, ``ts`` + ``rank``
  added), written by rank 0 only unless ``all_ranks=True``; flushed per record so a crashed run
  keeps everything up to the crash;
* :func:`log_metrics` — module-level convenience writing to ``$APNEAUQ_METRICS_JSONL`` if set.

The training callback that streams per-epoch logs is ``training.callbacks.JsonlLogger``.
"""
from __future__ import annotations

import json
import logging
import math
import os
import threading
import time
from typing import Any, Dict, Optional

_FMT = "%(asctime)s [rank %(rank)s] %(name)s %(levelname)s: %(message)s"


def _rank() -> int:
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:  # pragma: no cover - torch without distributed
        pass
    return int(os.environ.get("RANK", "0"))


class _RankFilter(logging.Filter):
    def filter(self, record: logging.LogRecord) -> bool:
        record.rank = _rank()
        return True


def get_logger(name: str = "apneauq", level: Optional[int] = None) -> logging.Logger:
    log = logging.getLogger(name)
    if not getattr(log, "_apneauq_configured", False):
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter(_FMT))
        h.addFilter(_RankFilter())
        log.addHandler(h)
        log.propagate = False
        log.setLevel(level if level is not None else getattr(logging, os.environ.get("APNEAUQ_LOG_LEVEL", "INFO")))
        log._apneauq_configured = True
    elif level is not None:
        log.setLevel(level)
    return log


def _jsonable(v: Any) -> Any:
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if hasattr(v, "item") and callable(v.item) and getattr(v, "ndim", 0) == 0:
        v = v.item()
    if isinstance(v, float) and not math.isfinite(v):
        return str(v)
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if hasattr(v, "tolist"):
        return _jsonable(v.tolist())
    return str(v)


class JsonlWriter:
    def __init__(self, path: str, all_ranks: bool = False):
        self.path = path
        self.enabled = all_ranks or _rank() == 0
        self._lock = threading.Lock()
        if self.enabled:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)

    def write(self, record: Dict[str, Any], **extra) -> None:
        if not self.enabled:
            return
        rec = {"ts": round(time.time(), 3), "rank": _rank()}
        rec.update(_jsonable(record))
        rec.update(_jsonable(extra))
        line = json.dumps(rec, sort_keys=False)
        with self._lock, open(self.path, "a") as f:
            f.write(line + "\n")
            f.flush()

    @staticmethod
    def read(path: str):
        with open(path) as f:
            return [json.loads(x) for x in f if x.strip()]


_DEFAULT: Optional[JsonlWriter] = None


def log_metrics(record: Dict[str, Any], **extra) -> None:
    """Write to ``$APNEAUQ_METRICS_JSONL`` (no-op when unset)."""
    global _DEFAULT
    path = os.environ.get("APNEAUQ_METRICS_JSONL")
    if not path:
        return
    if _DEFAULT is None or _DEFAULT.path != path:
        _DEFAULT = JsonlWriter(path)
    _DEFAULT.write(record, **extra)
