"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.analyze_de_patient_level`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import analyze_de_patient_level
from ..parallel.ensemble import load_ensemble  # noqa: F401
from ..uq.drivers import evaluate_deep_ensemble  # noqa: F401

if __name__ == "__main__":
    analyze_de_patient_level()
