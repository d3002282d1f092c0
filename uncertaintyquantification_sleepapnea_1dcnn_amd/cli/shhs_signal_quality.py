"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.shhs_signal_quality`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import shhs_signal_quality
from ..data.cohort import analyze_signal_quality  # noqa: F401

if __name__ == "__main__":
    shhs_signal_quality()
