"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.train_deep_ensemble_cnns`` (see commands.py)."""
from .commands import train_deep_ensemble_cnns

if __name__ == "__main__":
    train_deep_ensemble_cnns()
