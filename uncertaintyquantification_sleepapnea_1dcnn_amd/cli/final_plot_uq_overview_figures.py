"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.final_plot_uq_overview_figures`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import final_plot_uq_overview_figures
from ..analysis.figures import load_data  # noqa: F401

if __name__ == "__main__":
    final_plot_uq_overview_figures()
