"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.shhs_cohort_analysis`` (see commands.py)."""
from .commands import shhs_cohort_analysis

if __name__ == "__main__":
    shhs_cohort_analysis()
