"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.hyperparameter_plot_mcd_or_de_pass_convergence`` (see commands.py)."""
from .commands import hyperparameter_plot_mcd_or_de_pass_convergence

if __name__ == "__main__":
    hyperparameter_plot_mcd_or_de_pass_convergence()
