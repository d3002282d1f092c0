"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.preprocess_shhs_raw`` (see commands.py)."""
from .commands import preprocess_shhs_raw

if __name__ == "__main__":
    preprocess_shhs_raw()
