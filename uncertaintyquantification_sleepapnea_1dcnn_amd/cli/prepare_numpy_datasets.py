"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.prepare_numpy_datasets`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import prepare_numpy_datasets
from ..data.prepare import prepare_final_datasets, reshape_flat_to_3d, standardize_per_window  # noqa: F401

if __name__ == "__main__":
    prepare_numpy_datasets()
