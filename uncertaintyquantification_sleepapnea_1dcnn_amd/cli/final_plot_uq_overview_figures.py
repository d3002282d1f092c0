"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.final_plot_uq_overview_figures`` (see commands.py)."""
from .commands import final_plot_uq_overview_figures

if __name__ == "__main__":
    final_plot_uq_overview_figures()
