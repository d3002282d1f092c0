"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.patient_accuracy_entropy_correlation`` (see commands.py)."""
from .commands import patient_accuracy_entropy_correlation

if __name__ == "__main__":
    patient_accuracy_entropy_correlation()
