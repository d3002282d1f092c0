"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.aggregate_patient_uq_metrics`` (see commands.py)."""
from .commands import aggregate_patient_uq_metrics

if __name__ == "__main__":
    aggregate_patient_uq_metrics()
