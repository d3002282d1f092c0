"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.analyze_mcd_patient_level`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import analyze_mcd_patient_level
from ..uq.drivers import evaluate_mc_dropout  # noqa: F401

if __name__ == "__main__":
    analyze_mcd_patient_level()
