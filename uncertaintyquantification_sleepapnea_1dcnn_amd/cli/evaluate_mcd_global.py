"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.evaluate_mcd_global`` (see commands.py)."""
from .commands import evaluate_mcd_global

if __name__ == "__main__":
    evaluate_mcd_global()
