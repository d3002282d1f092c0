"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.analyze_window_level_uncertainty`` (see commands.py)."""
from .commands import analyze_window_level_uncertainty

if __name__ == "__main__":
    analyze_window_level_uncertainty()
