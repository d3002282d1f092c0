"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.patient_accuracy_entropy_correlation`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import patient_accuracy_entropy_correlation
from ..analysis.stats import calculate_and_print_correlation  # noqa: F401

if __name__ == "__main__":
    patient_accuracy_entropy_correlation()
