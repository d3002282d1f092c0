"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.shhs_cohort_analysis`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import shhs_cohort_analysis
from ..data.cohort import analyze_cohort  # noqa: F401

if __name__ == "__main__":
    shhs_cohort_analysis()
