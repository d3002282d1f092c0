"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.prepare_numpy_datasets`` (see commands.py)."""
from .commands import prepare_numpy_datasets

if __name__ == "__main__":
    prepare_numpy_datasets()
