"""``AlarconCNN1D`` — the Keras-like model object of the framework.

API parity with what the reference scripts call on their ``tf.keras.Model``
(``al_1d_cnn_create_model`` at ``cnn_baseline_train.py:37``): ``model(x, training=...)``,
``predict``, ``fit``, ``evaluate``, ``get_weights`` / ``set_weights`` (38 Keras-ordered arrays),
``save`` / :func:`load_model`, ``summary``, ``count_params``.

Execution backends (MI355X-first):

* inference (``training=False`` / ``predict``, MC Dropout, Deep Ensembles) on the GPU runs, for the
  reference architecture, the fp32-faithful layer-wise engine (``ops/x3.py``: conv products as three
  fp16 MFMAs over hi/lo splits, fp32 accumulate -- the reference computes in fp32) by default, or with
  ``precision="bf16"`` the bf16 fused whole-network kernel (``ops/fused.py``); other architectures
  run the layer-wise bf16 kernels (``ops/generic.py``).  Packed weights are cached per weight version;
* training steps run the layer-wise HIP kernels (``ops/train_ops.py``; replayed from a captured
  HIP graph on a single device) with the Keras BatchNorm/Dropout/Adam semantics -- bf16 MFMA operands
  by default, or with ``train_precision="fp32"`` the reference's fp32 (fp32 activations and gradients,
  fp32-input MFMA convs: ``ops/generic_train.py``, ``csrc/gf32_conv.hip``) -- or fp32 autograd over the
  reference ops where no kernel exists (CPU);
* ``model(x, training=True)`` reproduces Keras exactly: dropout on, BatchNorm on the statistics of
  the batch passed in, moving averages updated as a side effect (the reference's MC Dropout
  quirk).
On the CPU everything runs the fp32 reference.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import _ext, fused
from . import reference as R
from .params import ParamStore
from .spec import ModelSpec


def _default_device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class AlarconCNN1D:
    def __init__(self, input_shape: Sequence[int] = (60, 4), spec: Optional[ModelSpec] = None, seed: int = 2025,
                 device=None, name: str = "Alarcon_1D_CNN_Model", params=None, pool: bool = False,
                 precision: Optional[str] = None, train_precision: Optional[str] = None):
        self.spec = spec if spec is not None else ModelSpec.with_input(input_shape, pool=pool)
        self.name = name
        self.seed = int(seed)
        # inference precision on the GPU: "fp32" (fp32-faithful engine where it exists) or "bf16"
        self.precision = precision or os.environ.get("APNEAUQ_PRECISION", "fp32")
        if self.precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        # training precision on the GPU: "bf16" (bf16 MFMA operands, fp32 accumulation / master weights) or
        # "fp32" (the reference's: fp32 activations and gradients, fp32-input MFMA convs, csrc/gf32_conv.hip)
        self.train_precision = train_precision or os.environ.get("APNEAUQ_TRAIN_PRECISION", "bf16")
        if self.train_precision not in ("fp32", "bf16"):
            raise ValueError("train_precision must be 'fp32' or 'bf16'")
        self.device = torch.device(device) if device is not None else _default_device()
        init = params if params is not None else R.init_params(self.spec, self.seed)
        self.store = ParamStore(self.spec, init, self.device)
        from ..training.optim import Adam

        self.optimizer = Adam(1e-3)
        self.loss = "binary_crossentropy"
        self.metrics_names = ["loss", "accuracy", "auc"]
        self.stop_training = False
        self.dp = None  # parallel.data_parallel.DPContext when training data-parallel
        self._blob = None
        self._blob_version = -1
        self._call_counter = 0
        self._train_step_counter = 0

    # ------------------------------------------------------------------ Keras-like surface
    def compile(self, optimizer=None, loss="binary_crossentropy", metrics=None):
        if optimizer is not None:
            self.optimizer = optimizer
        self.loss = loss
        return self

    @property
    def input_shape(self) -> Tuple[Optional[int], int, int]:
        return (None, self.spec.input_length, self.spec.input_channels)

    def count_params(self) -> int:
        return self.spec.num_params()[0]

    def get_weights(self) -> List[np.ndarray]:
        return self.store.get_weights()

    def set_weights(self, arrays) -> None:
        self.store.set_weights(arrays)

    @property
    def params(self):
        return self.store.as_dict()

    def snapshot(self):
        return self.store.snapshot()

    def restore(self, snap) -> None:
        self.store.restore(snap)

    def summary(self, print_fn=print) -> str:
        ch, ln = self.spec.channels(), self.spec.lengths()
        rows = [f'Model: "{self.name}"', "_" * 72, f"{'Layer (type)':<34}{'Output Shape':<22}{'Param #':>12}", "=" * 72]
        for i, b in enumerate(self.spec.blocks, start=1):
            rows.append(f"{f'conv1d_{i} (Conv1D)':<34}{str((None, ln[i - 1], b.filters)):<22}"
                        f"{b.kernel_size * ch[i - 1] * b.filters + b.filters:>12,}")
            rows.append(f"{f'batchnorm_{i} (BatchNormalization)':<34}{str((None, ln[i - 1], b.filters)):<22}{4 * b.filters:>12,}")
            if b.pool:
                rows.append(f"{f'maxpool_{i} (MaxPooling1D)':<34}{str((None, ln[i], b.filters)):<22}{0:>12}")
            rows.append(f"{f'dropout_{i} (Dropout)':<34}{str((None, ln[i], b.filters)):<22}{0:>12}")
        rows.append(f"{'global_avg_pooling_1d (GlobalAveragePooling1D)':<34}{str((None, ch[-1])):<22}{0:>12}")
        rows.append(f"{'output_layer (Dense)':<34}{str((None, 1)):<22}{ch[-1] + 1:>12,}")
        tot, tr = self.spec.num_params()
        rows += ["=" * 72, f"Total params: {tot:,}", f"Trainable params: {tr:,}", f"Non-trainable params: {tot - tr:,}",
                 "_" * 72]
        text = "\n".join(rows)
        if print_fn is not None:
            print_fn(text)
        return text

    def to(self, device) -> "AlarconCNN1D":
        self.device = torch.device(device)
        self.store = self.store.to(self.device)
        self._blob = None
        self._gpack = None
        self._x3m = None
        for attr in ("_train_ws", "_mcd_ws", "_train_graphs", "_gtrain_ws", "_gfwd_ws", "_gtrain_ws32", "_gfwd_ws32",
                     "_gtrain_graphs"):  # device workspaces / captured graphs
            if hasattr(self, attr):
                delattr(self, attr)
        if self.optimizer.m is not None:
            self.optimizer.m = self.optimizer.m.to(self.device)
            self.optimizer.v = self.optimizer.v.to(self.device)
        return self

    # ------------------------------------------------------------------ inference
    def _as_input(self, x) -> torch.Tensor:
        if isinstance(x, torch.Tensor):
            t = x.to(self.device, torch.float32)
        else:
            t = torch.as_tensor(np.asarray(x), dtype=torch.float32, device=self.device)
        if t.dim() != 3 or t.shape[1] != self.spec.input_length or t.shape[2] != self.spec.input_channels:
            raise ValueError(f"expected input (N, {self.spec.input_length}, {self.spec.input_channels}), got {tuple(t.shape)}")
        return t

    def uses_fused(self) -> bool:
        """The reference architecture on a GPU: the fused whole-network kernel."""
        return self.device.type == "cuda" and fused.supports(self.spec)

    def uses_generic(self) -> bool:
        """Any other supported architecture on a GPU: the layer-wise HIP kernels (ops/generic.py)."""
        from ..ops import generic

        return self.device.type == "cuda" and not fused.supports(self.spec) and generic.supports(self.spec)

    def uses_x3(self) -> bool:
        """Inference on the fp32-faithful engine (reference architecture, precision "fp32", GPU)."""
        from ..ops import x3

        return self.device.type == "cuda" and self.precision == "fp32" and x3.supports(self.spec)

    def uses_tiled_x3(self) -> bool:
        """Running-BN inference on the fp32 fused whole-network kernel (``csrc/fused_tiled_x3.hip``: the
        pooled ensemble_cnn members, the 30 s single-channel window; precision "fp32", GPU)."""
        return (self.device.type == "cuda" and self.precision == "fp32" and not fused.supports(self.spec)
                and fused.tiled_net(self.spec) is not None and os.environ.get("APNEAUQ_TILED_FUSED", "1") != "0")

    def x3_model(self):
        """The engine's packed view of this model (cached per weight version; the BN moving statistics
        are views of the store's tensors, so batch-statistics MC Dropout updates them in place)."""
        from ..ops import x3

        if getattr(self, "_x3m", None) is None or self._x3m_version != self.store.version:
            self._x3m = x3.X3Model(self.spec, [self.store.as_dict()], device=self.device)
            self._x3m_version = self.store.version
        return self._x3m

    def hip_infer(self, x: torch.Tensor, n_pass: int = 1, dropout: bool = False, seed: Optional[int] = None,
                  pass_offset: int = 0, window_offset: int = 0, logits: bool = False) -> torch.Tensor:
        """(n_pass, N) fp32 probabilities (or logits), BN on running statistics, on the engine chosen by
        ``precision``: fp32 (the fp32-faithful x3 engine for the reference architecture, the fp32-input
        MFMA layer-wise kernels for any other; ``x``'s fp32 values) or bf16 (``x`` rounded to bf16)."""
        if self.uses_x3():
            from ..ops import x3

            _ext.require()
            return x3.forward_running(self.x3_model(), x, n_pass=n_pass, dropout=dropout,
                                      seed=self.seed if seed is None else seed, pass_offset=pass_offset,
                                      window_offset=window_offset, logits=logits)[0]
        if self.precision == "fp32" and self.uses_generic():
            from ..ops import generic_train

            if not generic_train.supports_fp32(self.spec):
                import warnings

                warnings.warn(f"precision='fp32': no fp32 HIP kernels for {self.spec} (kernel sizes > 15); "
                              "inference runs on the bf16 layer-wise kernels", RuntimeWarning, stacklevel=2)
                return self.hip_forward(x.to(torch.bfloat16).contiguous(), n_pass=n_pass, dropout=dropout,
                                        seed=seed, pass_offset=pass_offset, window_offset=window_offset,
                                        logits=logits)
            _ext.require()
            if self.uses_tiled_x3():
                # the pooled ensemble_cnn members / the 30 s single-channel window: the fp16x3 fused
                # whole-network kernel (csrc/fused_tiled_x3.hip)
                return fused.tiled_x3_forward(x, self.fused_blob_x3(), self.spec, n_pass=n_pass, dropout=dropout,
                                              seed=self.seed if seed is None else seed, pass_offset=pass_offset,
                                              window_offset=window_offset, logits=logits)[0]
            # any other architecture at fp32: the fp16x3 layer-wise path
            # (ops/generic_train.py:forward_running_f32)
            from ..ops import generic_train

            _ext.require()
            return generic_train.forward_running_f32(self, x, n_pass=n_pass, dropout=dropout,
                                                     seed=self.seed if seed is None else seed,
                                                     pass_offset=pass_offset, window_offset=window_offset,
                                                     logits=logits)
        return self.hip_forward(x.to(torch.bfloat16).contiguous(), n_pass=n_pass, dropout=dropout, seed=seed,
                                pass_offset=pass_offset, window_offset=window_offset, logits=logits)

    def uses_hip(self) -> bool:
        """Inference (running-stat BN) runs on hand-written HIP kernels; warns once when it cannot."""
        if self.device.type != "cuda":
            return False
        if self.uses_fused() or self.uses_generic():
            return True
        fused.warn_unsupported(self.spec, "inference")
        return False

    def generic_pack(self):
        if getattr(self, "_gpack", None) is None or self._gpack_version != self.store.version:
            from ..ops import generic

            self._gpack = generic.pack(self.spec, self.store.as_dict())
            self._gpack_version = self.store.version
        return self._gpack

    def hip_forward(self, x_bf16: torch.Tensor, n_pass: int = 1, dropout: bool = False, seed: Optional[int] = None,
                    pass_offset: int = 0, window_offset: int = 0, logits: bool = False) -> torch.Tensor:
        """(n_pass, N) fp32 probabilities (or logits) with running-stat BN on the HIP kernels."""
        _ext.require()
        seed = self.seed if seed is None else seed
        if self.uses_fused():
            return fused.fused_forward(x_bf16, self.fused_blob(), self.spec, n_pass=n_pass, dropout=dropout, seed=seed,
                                       pass_offset=pass_offset, window_offset=window_offset, logits=logits)[0]
        from ..ops import generic

        return generic.forward(self.generic_pack(), self.spec, x_bf16, n_pass=n_pass, dropout=dropout, seed=seed,
                               pass_offset=pass_offset, window_offset=window_offset, logits=logits)

    def fused_blob_x3(self) -> torch.Tensor:
        """Packed fp16x3 parameters for the fp32 fused kernel (cached per weight version)."""
        if getattr(self, "_blob3", None) is None or self._blob3_version != self.store.version:
            self._blob3 = fused.pack_blob_x3(self.spec, self.store.as_dict()).unsqueeze(0)
            self._blob3_version = self.store.version
        return self._blob3

    def fused_blob(self) -> torch.Tensor:
        """Packed parameters for the fused HIP kernel (cached per weight version)."""
        if self._blob is None or self._blob_version != self.store.version:
            self._blob = fused.pack_blob(self.spec, self.store.as_dict()).unsqueeze(0)
            self._blob_version = self.store.version
        return self._blob

    def logits(self, x, training: bool = False, *, dropout: Optional[bool] = None,
               bn_batch_stats: Optional[bool] = None, update_moving: Optional[bool] = None, seed: Optional[int] = None,
               pass_id: Optional[int] = None, sample_ids=None) -> torch.Tensor:
        x = self._as_input(x)
        use_drop = training if dropout is None else dropout
        use_batch = training if bn_batch_stats is None else bn_batch_stats
        if not use_batch and self.uses_hip() and (sample_ids is None or not isinstance(sample_ids, torch.Tensor)):
            sid = 0 if sample_ids is None else int(sample_ids)
            out = self.hip_infer(x, n_pass=1, dropout=use_drop, seed=seed,
                                 pass_offset=0 if pass_id is None else pass_id, window_offset=sid, logits=True)
            return out[0].reshape(-1, 1)
        upd = use_batch if update_moving is None else update_moving
        with torch.no_grad():
            out = R.forward(self.spec, self.store.as_dict(), x, dropout=use_drop, bn_batch_stats=use_batch,
                            update_moving=upd, seed=self.seed if seed is None else seed,
                            pass_id=0 if pass_id is None else pass_id, return_logits=True,
                            sample_ids=sample_ids if isinstance(sample_ids, torch.Tensor) else None)
        if upd and use_batch:
            self.store.bump()
        return out

    def __call__(self, x, training: bool = False) -> torch.Tensor:
        """Keras ``model(x, training=...)``: returns (N, 1) fp32 probabilities on the model device.

        ``training=True`` draws a fresh dropout stream per call (pass id = call counter).
        """
        pass_id = None
        if training:
            pass_id = self._call_counter
            self._call_counter += 1
        return torch.sigmoid(self.logits(x, training=training, pass_id=pass_id))

    def predict(self, x, batch_size: int = 32, verbose: int = 0) -> np.ndarray:
        """Inference-mode probabilities (N, 1) as float32 NumPy (``model.predict``).

        The fused kernel processes the whole array in one launch; ``batch_size`` only bounds the
        CPU path's memory (results are independent of it).
        """
        x = self._as_input(x)
        if self.uses_hip():
            return torch.sigmoid(self.logits(x)).cpu().numpy()
        outs = []
        step = max(int(batch_size), 4096)
        for s in range(0, x.shape[0], step):
            outs.append(torch.sigmoid(self.logits(x[s: s + step])).cpu().numpy())
        return np.concatenate(outs) if outs else np.zeros((0, 1), np.float32)

    # ------------------------------------------------------------------ training
    def train_step(self, x, y, return_probs: bool = False, grad_allreduce=None, dp_step=None):
        """One optimizer step on a batch (Keras training semantics); returns the summed BCE."""
        from ..training import step as tstep

        loss_sum, probs = tstep.train_step(self, self._as_input(x), torch.as_tensor(y, device=self.device).float(),
                                           grad_allreduce=grad_allreduce, dp_step=dp_step)
        self._train_step_counter += 1
        self.store.bump()
        if return_probs:
            return loss_sum, probs
        return float(loss_sum)

    def fit(self, x, y, batch_size: int = 32, epochs: int = 1, verbose: int = 1, callbacks=None,
            validation_split: float = 0.0, validation_data=None, shuffle: bool = True, **kw):
        from ..training.trainer import fit as _fit

        return _fit(self, x, y, batch_size=batch_size, epochs=epochs, verbose=verbose, callbacks=callbacks,
                    validation_split=validation_split, validation_data=validation_data, shuffle=shuffle, **kw)

    def evaluate(self, x, y, batch_size: int = 32, verbose: int = 0):
        from ..training.trainer import evaluate_arrays

        X = self._as_input(x)
        Y = torch.as_tensor(np.asarray(y), dtype=torch.float32, device=self.device)
        return list(evaluate_arrays(self, X, Y, max(batch_size, 1024)))

    # ------------------------------------------------------------------ persistence
    def save(self, path: str, include_optimizer: bool = False) -> str:
        from ..utils.checkpoint import save_weights

        opt = None
        if include_optimizer and self.optimizer.m is not None:
            opt = {"m": self.optimizer.m.cpu().numpy(), "v": self.optimizer.v.cpu().numpy(),
                   "iterations": np.array(self.optimizer.iterations)}
        return save_weights(path, self.spec, self.get_weights(), self.name, extra={"seed": self.seed}, opt_state=opt)


def load_model(path: str, device=None) -> AlarconCNN1D:
    """Load a checkpoint written by :meth:`AlarconCNN1D.save` (safe: no code is deserialised)."""
    from ..utils.checkpoint import load_weights

    spec, arrays, cfg, opt = load_weights(path)
    m = AlarconCNN1D(spec=spec, seed=int(cfg.get("extra", {}).get("seed", 2025)), device=device,
                     name=cfg.get("name", "Alarcon_1D_CNN_Model"), params=R.params_from_list(spec, arrays))
    if opt:
        m.optimizer.iterations = int(opt["iterations"])
        m.optimizer.m = torch.from_numpy(opt["m"]).to(m.device)
        m.optimizer.v = torch.from_numpy(opt["v"]).to(m.device)
    return m


def al_1d_cnn_create_model(input_shape: Sequence[int] = (60, 4), seed: int = 2025, device=None) -> AlarconCNN1D:
    """Factory with the reference's name (``cnn_baseline_train.py:37``); returns a compiled model."""
    return AlarconCNN1D(input_shape=input_shape, seed=seed, device=device).compile()
