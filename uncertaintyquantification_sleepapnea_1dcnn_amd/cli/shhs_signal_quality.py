"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.shhs_signal_quality`` (see commands.py)."""
from .commands import shhs_signal_quality

if __name__ == "__main__":
    shhs_signal_quality()
