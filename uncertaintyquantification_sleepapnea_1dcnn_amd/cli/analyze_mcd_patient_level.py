"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.analyze_mcd_patient_level`` (see commands.py)."""
from .commands import analyze_mcd_patient_level

if __name__ == "__main__":
    analyze_mcd_patient_level()
