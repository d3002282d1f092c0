"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.cnn_baseline_train`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import cnn_baseline_train
from ..models.cnn import al_1d_cnn_create_model  # noqa: F401
from ..training.experiment import run_cnn_experiment  # noqa: F401

if __name__ == "__main__":
    cnn_baseline_train()
