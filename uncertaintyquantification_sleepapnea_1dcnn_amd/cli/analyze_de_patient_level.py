"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.analyze_de_patient_level`` (see commands.py)."""
from .commands import analyze_de_patient_level

if __name__ == "__main__":
    analyze_de_patient_level()
