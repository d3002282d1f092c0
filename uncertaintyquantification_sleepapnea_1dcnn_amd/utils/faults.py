"""Fault injection for recovery tests (SURVEY §5 "Failure detection / elastic recovery").

The reference's recovery story is member-granularity skip-if-exists
(``train_deep_ensemble_cnns.py:130-132``) plus print-and-continue ``try/except`` blocks.  The
framework keeps member granularity as the unit of recovery (``parallel/ensemble.py``) and
epoch granularity inside a member (``training.callbacks.BackupAndRestore``); this module lets a
test kill a process at a named site to prove both:

    APNEAUQ_FAULT="ensemble.before_save:member=2"      # hard-exit the process training member 2
    APNEAUQ_FAULT="fit.epoch_end:epoch=1;rank=0"       # hard-exit rank 0 after epoch index 1

Coordinates not named in the spec match anything.  The process exits with ``os._exit`` (no
cleanup, no exception handlers — like a killed rank) and code ``APNEAUQ_FAULT_CODE`` (default 17).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

FAULT_ENV = "APNEAUQ_FAULT"


def _parse(spec: str) -> Tuple[str, Dict[str, str]]:
    site, _, rest = spec.partition(":")
    coords = {}
    for kv in filter(None, rest.replace(",", ";").split(";")):
        k, _, v = kv.partition("=")
        coords[k.strip()] = v.strip()
    return site.strip(), coords


def armed(site: str, **coords) -> bool:
    spec: Optional[str] = os.environ.get(FAULT_ENV)
    if not spec:
        return False
    for one in spec.split("|"):
        s, want = _parse(one)
        if s != site:
            continue
        if "rank" not in coords:
            coords = dict(coords, rank=os.environ.get("RANK", "0"))
        if all(str(coords.get(k)) == v for k, v in want.items()):
            return True
    return False


def maybe_fail(site: str, **coords) -> None:
    if armed(site, **coords):
        os._exit(int(os.environ.get("APNEAUQ_FAULT_CODE", "17")))
