"""One run configuration for every stage (SURVEY §5 "Config / flag system", quirk Q8).

The reference scatters its settings over module constants and seven argparse blocks, and the
stages disagree on file and directory names (``prepare_numpy_datasets.py:48`` writes
``./processed_datasets2``; ``cnn_baseline_train.py:22`` reads ``./final_processed_datasets``;
``train_deep_ensemble_cnns.py:15`` and the UQ drivers read ``./processed_datasets``).  Here one
dataclass carries the paths and the experiment constants; the CLI entry points keep the
reference's flag names and defaults and only fall back to this object.

Load order: defaults < JSON/YAML file (``APNEAUQ_CONFIG`` or explicit path) < ``APNEAUQ_<FIELD>``
environment variables < explicit keyword overrides.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Any, Dict, Optional


@dataclasses.dataclass
class RunConfig:
    # ---- paths (reference defaults)
    edf_folder: str = ""
    xml_folder: str = ""
    raw_csv: str = "./SHHS2_ID_all_60.csv"
    processed_dir: str = "./final_processed_datasets"
    model_path: str = "./alarcon_cnn_model.keras"
    mcd_model_path: str = "./AlCNN1D_no_pool.keras"
    ensemble_dir: str = "./models/ensemble_cnn_no_pool"
    output_dir: str = "./uq_results"
    plot_dir: str = "./uq_plots"
    # ---- experiment constants
    seed: int = 2025
    mcd_passes: int = 50            # analyze_mcd_patient_level.py:21
    de_members: int = 5             # analyze_de_patient_level.py:20 (20 in evaluate_de_global.py:11)
    n_bootstrap: int = 100          # analyze_mcd_patient_level.py:23
    bn_mode: str = "batch"          # MC-Dropout BN semantics: "batch" (reference parity) | "running"
    epochs: int = 30                # cnn_baseline_train.py:31 (50 for the ensemble trainer)
    batch_size: int = 1024
    patience: int = 5
    validation_split: float = 0.1
    learning_rate: float = 1e-3
    # ---- model / numerics
    input_length: int = 60
    input_channels: int = 4
    pool: bool = False              # opt-in MaxPool1D per block
    dtype: str = "bf16"             # compute dtype of the HIP kernels (fp32 accumulation)
    deterministic: bool = False     # fixed-order reductions in the HIP training step (bitwise-reproducible
                                    # weights; ops/train_ops.set_deterministic, env APNEAUQ_DETERMINISTIC)
    # ---- distribution
    world_size: int = 1
    backend: str = "auto"           # "nccl" (RCCL) on GPUs, "gloo" on CPU

    def __post_init__(self):
        if self.bn_mode not in ("batch", "running"):
            raise ValueError(f"bn_mode must be 'batch' or 'running', got {self.bn_mode!r}")
        if self.dtype not in ("bf16", "fp32"):
            raise ValueError(f"dtype must be 'bf16' or 'fp32', got {self.dtype!r}")

    # ------------------------------------------------------------------ io
    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def to_json(self, path: Optional[str] = None) -> str:
        s = json.dumps(self.to_dict(), indent=1, sort_keys=True)
        if path:
            with open(path, "w") as f:
                f.write(s)
        return s

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RunConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        unknown = set(d) - names
        if unknown:
            raise KeyError(f"unknown config keys: {sorted(unknown)}")
        return cls(**d)

    @classmethod
    def load(cls, path: Optional[str] = None, env: bool = True, **overrides) -> "RunConfig":
        d: Dict[str, Any] = {}
        path = path or (os.environ.get("APNEAUQ_CONFIG") if env else None)
        if path:
            with open(path) as f:
                if path.endswith((".yaml", ".yml")):
                    import yaml

                    d.update(yaml.safe_load(f) or {})
                else:
                    d.update(json.load(f))
        if env:
            for fld in dataclasses.fields(cls):
                v = os.environ.get("APNEAUQ_" + fld.name.upper())
                if v is not None:
                    d[fld.name] = _coerce(v, fld.type)
        d.update(overrides)
        return cls.from_dict(d)

    # ------------------------------------------------------------------ helpers
    def spec(self):
        from ..models.spec import DEFAULT_BLOCKS, BlockSpec, ModelSpec

        return ModelSpec(input_length=self.input_length, input_channels=self.input_channels,
                         blocks=tuple(BlockSpec(f, k, p, self.pool) for f, k, p in DEFAULT_BLOCKS))

    def processed(self, name: str) -> str:
        return os.path.join(self.processed_dir, name)


def _coerce(v: str, typ) -> Any:
    t = typ if isinstance(typ, str) else getattr(typ, "__name__", str(typ))
    if t == "bool":
        return v.strip().lower() in ("1", "true", "yes", "on")
    if t == "int":
        return int(v)
    if t == "float":
        return float(v)
    return v
