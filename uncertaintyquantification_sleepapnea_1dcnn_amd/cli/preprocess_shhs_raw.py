"""CLI: ``python -m uncertaintyquantification_sleepapnea_1dcnn_amd.cli.preprocess_shhs_raw`` (see commands.py).

Also exports the reference script's functions under their reference names."""
from .commands import preprocess_shhs_raw
from ..data.annotations import calculate_sleep_time, parse_xml_annotations  # noqa: F401
from ..data.preprocess import (check_artifacts_and_missing_values, get_edf_channels, main,  # noqa: F401
                               process_all_files, process_single_file, remove_artifacts, resample_signals,
                               segment_and_label_edf_data)

if __name__ == "__main__":
    preprocess_shhs_raw()
