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
