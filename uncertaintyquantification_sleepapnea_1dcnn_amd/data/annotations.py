"""NSRR XML annotation parsing and the recording-duration gate.

``parse_xml_annotations`` follows ``preprocess_shhs_raw.py:169-190``: iterate
``ScoredEvents/ScoredEvent`` and STOP at the first ``Stages|Stages`` event, emitting
``{event_type, event_concept, start, duration}``.

``calculate_sleep_time`` implements the intended rule of ``preprocess_shhs_raw.py:75-96``
(duration of the "Recording Start Time" event >= 300 min) with the key names the parser actually
emits.  The reference looks up ``"EventConcept"``/``"Duration"`` and therefore raises KeyError
on every file, which its per-file ``try/except`` turns into "excluded" (SURVEY Q7).  Set
``reference_keys=True`` to reproduce that behaviour.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET
from typing import Dict, List, Optional

APNEA_EVENTS = ("Obstructive apnea|Obstructive Apnea", "Hypopnea|Hypopnea")


def _text(el, tag) -> Optional[str]:
    c = el.find(tag)
    return c.text if c is not None else None


def parse_xml_annotations(xml_file_path: str) -> List[Dict]:
    root = ET.parse(xml_file_path).getroot()
    events = []
    for ev in root.findall("ScoredEvents/ScoredEvent"):
        et = _text(ev, "EventType")
        if et == "Stages|Stages":
            break
        start = _text(ev, "Start")
        dur = _text(ev, "Duration")
        events.append({"event_type": et, "event_concept": _text(ev, "EventConcept"),
                       "start": float(start) if start is not None else None,
                       "duration": float(dur) if dur is not None else None})
    return events


def calculate_sleep_time(events: List[Dict], min_sleep_time: float = 300 * 60, reference_keys: bool = False,
                         verbose: bool = True) -> bool:
    kc, kd = ("EventConcept", "Duration") if reference_keys else ("event_concept", "duration")
    ev = next((e for e in events if e[kc] == "Recording Start Time"), None)
    total = ev[kd] if ev else 0
    if verbose:
        print(f"Total sleep time (based on Recording Start Time): {total}")
    return (total or 0) >= min_sleep_time


def write_xml_annotations(path: str, events: List[Dict], stages: bool = True) -> str:
    """Write an NSRR-style annotation file (used for synthetic test recordings)."""
    root = ET.Element("PSGAnnotation")
    se = ET.SubElement(root, "ScoredEvents")
    for e in events:
        x = ET.SubElement(se, "ScoredEvent")
        ET.SubElement(x, "EventType").text = e.get("event_type", "Respiratory|Respiratory")
        ET.SubElement(x, "EventConcept").text = e["event_concept"]
        ET.SubElement(x, "Start").text = str(e["start"])
        ET.SubElement(x, "Duration").text = str(e["duration"])
    if stages:
        x = ET.SubElement(se, "ScoredEvent")
        ET.SubElement(x, "EventType").text = "Stages|Stages"
        ET.SubElement(x, "EventConcept").text = "Wake|0"
        ET.SubElement(x, "Start").text = "0"
        ET.SubElement(x, "Duration").text = "30"
    ET.ElementTree(root).write(path)
    return path
