"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.window_uncertainty_vs_correctness_mannwhitney`` (see commands.py)."""
from .commands import window_uncertainty_vs_correctness_mannwhitney

if __name__ == "__main__":
    window_uncertainty_vs_correctness_mannwhitney()
