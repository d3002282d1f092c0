"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.evaluate_de_global`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import evaluate_de_global
from ..parallel.ensemble import load_ensemble_prefix as load_ensemble  # noqa: F401  (reference signature)
from ..uq.drivers import evaluate_ensemble  # noqa: F401

if __name__ == "__main__":
    evaluate_de_global()
