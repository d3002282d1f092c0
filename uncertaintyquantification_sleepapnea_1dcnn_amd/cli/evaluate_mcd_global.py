"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.evaluate_mcd_global`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import evaluate_mcd_global
from ..uq.drivers import evaluate_mc_dropout_global as evaluate_mc_dropout  # noqa: F401  (reference signature)

if __name__ == "__main__":
    evaluate_mcd_global()
