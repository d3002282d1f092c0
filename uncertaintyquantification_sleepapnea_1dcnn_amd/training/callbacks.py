"""Keras-semantics callbacks: History and EarlyStopping(restore_best_weights).

EarlyStopping mirrors Keras 2.12 (the version the reference pins, ``README.md:79``) as used at
``cnn_baseline_train.py:204-208`` and ``train_deep_ensemble_cnns.py:150-154``:
``wait`` increments every epoch and resets on an improvement of the monitored value; training
stops when ``wait >= patience`` (never after epoch 0); best weights are captured in device
memory and restored ONLY when the stop triggers — not at the natural end of training.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional


class Callback:
    model = None

    def set_model(self, model) -> None:
        self.model = model

    def on_train_begin(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass


class History(Callback):
    def __init__(self):
        self.history: Dict[str, List[float]] = {}
        self.epoch: List[int] = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class EarlyStopping(Callback):
    def __init__(self, monitor: str = "val_loss", min_delta: float = 0.0, patience: int = 0, verbose: int = 0,
                 mode: str = "auto", baseline: Optional[float] = None, restore_best_weights: bool = False,
                 start_from_epoch: int = 0):
        self.monitor = monitor
        self.patience = patience
        self.verbose = verbose
        self.baseline = baseline
        self.min_delta = abs(min_delta)
        self.restore_best_weights = restore_best_weights
        self.start_from_epoch = start_from_epoch
        if mode not in ("auto", "min", "max"):
            mode = "auto"
        if mode == "max" or (mode == "auto" and ("acc" in monitor or monitor.endswith("auc"))):
            self._better = lambda a, b: a - self.min_delta > b
            self._init = -math.inf
        else:
            self._better = lambda a, b: a + self.min_delta < b
            self._init = math.inf
        self.wait = 0
        self.stopped_epoch = 0
        self.best = self._init
        self.best_weights = None
        self.best_epoch = 0

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.stopped_epoch = 0
        self.best = self._init
        self.best_weights = None
        self.best_epoch = 0

    def on_epoch_end(self, epoch, logs=None):
        current = (logs or {}).get(self.monitor)
        if current is None or epoch < self.start_from_epoch:
            return
        if self.restore_best_weights and self.best_weights is None:
            self.best_weights = self.model.snapshot()  # first epoch: in case nothing ever improves
        self.wait += 1
        if self._better(current, self.best):
            self.best = current
            self.best_epoch = epoch
            if self.restore_best_weights:
                self.best_weights = self.model.snapshot()
            if self.baseline is None or self._better(current, self.baseline):
                self.wait = 0
            return
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            self.model.stop_training = True
            if self.restore_best_weights and self.best_weights is not None:
                if self.verbose > 0:
                    print(f"Restoring model weights from the end of the best epoch: {self.best_epoch + 1}.")
                self.model.restore(self.best_weights)

    def on_train_end(self, logs=None):
        if self.stopped_epoch > 0 and self.verbose > 0:
            print(f"Epoch {self.stopped_epoch + 1}: early stopping")


class JsonlLogger(Callback):
    """Stream per-epoch logs (loss, accuracy, auc, val_*) as JSON lines (SURVEY §5 observability).

    The reference persists nothing of its ``History`` (``train_deep_ensemble_cnns.py:171``)."""

    def __init__(self, path: str, run: Optional[str] = None, all_ranks: bool = False):
        from ..utils.logging import JsonlWriter

        self.writer = JsonlWriter(path, all_ranks=all_ranks)
        self.run = run
        self._t0 = None

    def on_train_begin(self, logs=None):
        import time

        self._t0 = time.time()
        self.writer.write({"event": "train_begin", "run": self.run, "model": getattr(self.model, "name", None)})

    def on_epoch_end(self, epoch, logs=None):
        import time

        self.writer.write({"event": "epoch", "run": self.run, "epoch": epoch, "elapsed_s": time.time() - self._t0, **(logs or {})})

    def on_train_end(self, logs=None):
        self.writer.write({"event": "train_end", "run": self.run})


class BackupAndRestore(Callback):
    """Epoch-granularity fault tolerance (Keras ``callbacks.BackupAndRestore`` semantics).

    After every epoch the weights, the Adam state (m, v, iterations), the dropout step counter and
    the epoch index are written atomically to ``backup_dir``.  When a training run starts and a
    backup exists, it is restored and ``fit`` resumes at the next epoch (its shuffling generator is
    fast-forwarded, so the resumed run sees the same batches as an uninterrupted one).  The backup
    is deleted when training ends normally.  As in Keras, other callbacks' state (e.g.
    EarlyStopping's patience counter) is not part of the backup.
    """

    FILE = "backup.npz"

    def __init__(self, backup_dir: str, delete_checkpoint: bool = True):
        self.backup_dir = backup_dir
        self.delete_checkpoint = delete_checkpoint

    @property
    def path(self) -> str:
        import os

        return os.path.join(self.backup_dir, self.FILE)

    def on_train_begin(self, logs=None):
        import os

        import numpy as np
        import torch

        from ..utils.checkpoint import load_weights

        if not os.path.exists(self.path):
            return
        spec, arrays, cfg, opt = load_weights(self.path)
        m = self.model
        m.set_weights(arrays)
        if opt:
            m.optimizer.iterations = int(opt["iterations"])
            m.optimizer.m = torch.from_numpy(np.array(opt["m"])).to(m.device)
            m.optimizer.v = torch.from_numpy(np.array(opt["v"])).to(m.device)
        extra = cfg.get("extra", {})
        m._train_step_counter = int(extra.get("train_step_counter", 0))
        m._resume_epoch = int(extra["epoch"]) + 1

    def on_epoch_end(self, epoch, logs=None):
        import os

        import numpy as np

        from ..utils.checkpoint import save_weights

        m = self.model
        dp = getattr(m, "dp", None)
        if dp is not None and dp.rank != 0:
            return  # one writer per data-parallel group; every rank restores from it
        os.makedirs(self.backup_dir, exist_ok=True)
        opt = None
        if m.optimizer.m is not None:
            opt = {"m": m.optimizer.m.cpu().numpy(), "v": m.optimizer.v.cpu().numpy(),
                   "iterations": np.array(m.optimizer.iterations)}
        save_weights(self.path, m.spec, m.get_weights(), m.name,
                     extra={"seed": m.seed, "epoch": int(epoch), "train_step_counter": int(m._train_step_counter)},
                     opt_state=opt)

    def on_train_end(self, logs=None):
        import os

        dp = getattr(self.model, "dp", None)
        if dp is not None and dp.rank != 0:
            return
        if self.delete_checkpoint and os.path.exists(self.path):
            os.remove(self.path)
            try:
                os.rmdir(self.backup_dir)  # only if empty
            except OSError:
                pass
