"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.hyperparameter_plot_mcd_or_de_pass_convergence`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import hyperparameter_plot_mcd_or_de_pass_convergence
from ..analysis.figures import plot_variance_convergence  # noqa: F401

if __name__ == "__main__":
    hyperparameter_plot_mcd_or_de_pass_convergence()
