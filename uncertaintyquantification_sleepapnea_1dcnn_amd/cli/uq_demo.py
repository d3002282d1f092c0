"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.uq_demo`` (see commands.py)."""
from .commands import uq_demo

if __name__ == "__main__":
    uq_demo()
