"""Architecture specification of the Alarcón 1D-CNN and its Keras-ordered weight layout.

The reference builds the network twice (``models/cnn_baseline_train.py:37-104`` and
``models/train_deep_ensemble_cnns.py:25-77``) as a Keras ``Sequential`` of six
``Conv1D(relu, same) -> BatchNormalization -> Dropout`` blocks followed by
``GlobalAveragePooling1D -> Dense(1, sigmoid)``.  Here the architecture is plain data
(:class:`ModelSpec`) so that the HIP kernels, the CPU reference, the checkpoint format and
the tests all derive from one description.

Weight layout (``get_weights`` order, 38 arrays for the default spec):
per conv block ``[kernel (k, Cin, Cout), bias (Cout,)]`` then per BN
``[gamma, beta, moving_mean, moving_variance]`` and finally the dense
``[kernel (C_last, 1), bias (1,)]``.
"""
from __future__ import annotations

import dataclasses
import json
from typing import List, Sequence, Tuple

# (filters, kernel_size, dropout_rate) -- cnn_baseline_train.py:59-86
DEFAULT_BLOCKS: Tuple[Tuple[int, int, float], ...] = (
    (128, 7, 0.3),
    (192, 5, 0.3),
    (224, 3, 0.4),
    (96, 7, 0.2),
    (256, 9, 0.3),
    (96, 9, 0.5),
)

# Keras 2.12 defaults that fix the semantics ("Keras 2.12 defaults")
BN_EPSILON = 1e-3
BN_MOMENTUM = 0.99
ADAM_EPSILON = 1e-7


@dataclasses.dataclass(frozen=True)
class BlockSpec:
    filters: int
    kernel_size: int
    dropout: float
    pool: bool = False  # opt-in MaxPool1D(2, valid) after BN, before Dropout


@dataclasses.dataclass(frozen=True)
class ModelSpec:
    """Architecture of the Alarcón 1D-CNN.

    ``input_length``/``input_channels`` default to the reference's (60, 4) windows
    (``prepare_numpy_datasets.py:53-55``); the north-star "30 s single-channel" shape is
    ``ModelSpec(input_length=30, input_channels=1)``.
    """

    input_length: int = 60
    input_channels: int = 4
    blocks: Tuple[BlockSpec, ...] = tuple(BlockSpec(f, k, p) for f, k, p in DEFAULT_BLOCKS)
    bn_epsilon: float = BN_EPSILON
    bn_momentum: float = BN_MOMENTUM

    # ------------------------------------------------------------------ shapes
    @property
    def num_blocks(self) -> int:
        return len(self.blocks)

    def channels(self) -> List[int]:
        """Channel count entering each block, plus the final one: [C_in, c1, ..., c6]."""
        return [self.input_channels] + [b.filters for b in self.blocks]

    def lengths(self) -> List[int]:
        """Sequence length entering each block, plus the final one."""
        out = [self.input_length]
        for b in self.blocks:
            out.append(out[-1] // 2 if b.pool else out[-1])
        return out

    @property
    def has_pool(self) -> bool:
        return any(b.pool for b in self.blocks)

    @property
    def final_channels(self) -> int:
        return self.blocks[-1].filters

    def weight_names(self) -> List[str]:
        """Keras-style variable names in ``get_weights`` order."""
        names = []
        for i in range(1, self.num_blocks + 1):
            names += [f"conv1d_{i}/kernel", f"conv1d_{i}/bias"]
            names += [f"batchnorm_{i}/gamma", f"batchnorm_{i}/beta",
                      f"batchnorm_{i}/moving_mean", f"batchnorm_{i}/moving_variance"]
        names += ["output_layer/kernel", "output_layer/bias"]
        return names

    def weight_shapes(self) -> List[Tuple[int, ...]]:
        ch = self.channels()
        shapes: List[Tuple[int, ...]] = []
        for i, b in enumerate(self.blocks):
            shapes += [(b.kernel_size, ch[i], b.filters), (b.filters,)]
            shapes += [(b.filters,)] * 4
        shapes += [(self.final_channels, 1), (1,)]
        return shapes

    def trainable_mask(self) -> List[bool]:
        m: List[bool] = []
        for _ in self.blocks:
            m += [True, True, True, True, False, False]
        m += [True, True]
        return m

    def num_params(self) -> Tuple[int, int]:
        """(total, trainable) parameter counts; 853,441 / 851,457 for the default spec."""
        tot = tr = 0
        for shp, t in zip(self.weight_shapes(), self.trainable_mask()):
            n = 1
            for s in shp:
                n *= s
            tot += n
            tr += n if t else 0
        return tot, tr

    def forward_macs(self) -> int:
        """Multiply-accumulates per window of one forward pass (50.90 M for the default spec)."""
        ch, ln = self.channels(), self.lengths()
        macs = 0
        for i, b in enumerate(self.blocks):
            macs += ln[i] * b.kernel_size * ch[i] * b.filters
        return macs + self.final_channels

    # ------------------------------------------------------------------ (de)serialisation
    def to_dict(self) -> dict:
        return {
            "input_length": self.input_length,
            "input_channels": self.input_channels,
            "blocks": [[b.filters, b.kernel_size, b.dropout, b.pool] for b in self.blocks],
            "bn_epsilon": self.bn_epsilon,
            "bn_momentum": self.bn_momentum,
        }

    @classmethod
    def from_dict(cls, d: dict) -> "ModelSpec":
        blocks = tuple(BlockSpec(int(f), int(k), float(p), bool(pl)) for f, k, p, pl in d["blocks"])
        return cls(int(d["input_length"]), int(d["input_channels"]), blocks,
                   float(d.get("bn_epsilon", BN_EPSILON)), float(d.get("bn_momentum", BN_MOMENTUM)))

    def to_json(self) -> str:
        return json.dumps(self.to_dict())

    @classmethod
    def with_input(cls, input_shape: Sequence[int], pool: bool = False) -> "ModelSpec":
        blocks = tuple(BlockSpec(f, k, p, pool) for f, k, p in DEFAULT_BLOCKS)
        return cls(int(input_shape[0]), int(input_shape[1]), blocks)


DEFAULT_SPEC = ModelSpec()
