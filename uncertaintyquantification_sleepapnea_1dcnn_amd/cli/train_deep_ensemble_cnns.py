"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.train_deep_ensemble_cnns`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import train_deep_ensemble_cnns
from ..models.cnn import al_1d_cnn_create_model  # noqa: F401
from .commands import reference_train_ensemble as train_ensemble  # noqa: F401  (reference signature)

if __name__ == "__main__":
    train_deep_ensemble_cnns()
