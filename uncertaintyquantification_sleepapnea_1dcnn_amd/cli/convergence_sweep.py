"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.convergence_sweep`` (see commands.py)."""
from .commands import convergence_sweep

if __name__ == "__main__":
    convergence_sweep()
