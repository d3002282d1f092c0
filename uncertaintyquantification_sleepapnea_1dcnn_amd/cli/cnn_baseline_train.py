"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.cnn_baseline_train`` (see commands.py)."""
from .commands import cnn_baseline_train

if __name__ == "__main__":
    cnn_baseline_train()
