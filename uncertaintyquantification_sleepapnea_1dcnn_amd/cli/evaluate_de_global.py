"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.evaluate_de_global`` (see commands.py)."""
from .commands import evaluate_de_global

if __name__ == "__main__":
    evaluate_de_global()
