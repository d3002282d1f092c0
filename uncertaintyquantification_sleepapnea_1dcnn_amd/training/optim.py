"""Keras-2.12-exact Adam on a flat parameter buffer (HIP multi-tensor kernel on the GPU).

``tf.keras.optimizers.Adam(learning_rate=0.001)`` (``cnn_baseline_train.py:100``) with its
defaults beta_1=0.9, beta_2=0.999, epsilon=1e-7 and the update
``p -= lr*sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)`` (epsilon outside the bias correction).
"""
from __future__ import annotations

import math
from typing import Dict

import torch

from ..models.spec import ADAM_EPSILON
from ..ops import _ext


class Adam:
    def __init__(self, learning_rate: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = ADAM_EPSILON):
        self.learning_rate = float(learning_rate)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)
        self.iterations = 0
        self.m = None
        self.v = None

    def get_config(self) -> Dict[str, float]:
        return {"learning_rate": self.learning_rate, "beta_1": self.beta_1, "beta_2": self.beta_2,
                "epsilon": self.epsilon}

    def _ensure(self, flat: torch.Tensor) -> None:
        if self.m is None or self.m.shape != flat.shape or self.m.device != flat.device:
            self.m = torch.zeros_like(flat)
            self.v = torch.zeros_like(flat)

    def alpha(self) -> float:
        t = self.iterations + 1
        return self.learning_rate * math.sqrt(1.0 - self.beta_2 ** t) / (1.0 - self.beta_1 ** t)

    @torch.no_grad()
    def step(self, flat: torch.Tensor, grad: torch.Tensor, grad_scale: float = 1.0, counters=None) -> None:
        """``counters`` (int32 GPU tensor [.., iterations]): the bias correction is computed on the
        device from the iteration counter -- the arithmetic of a captured (HIP-graph) step, so eager
        and graphed steps give bitwise-identical weights."""
        self._ensure(flat)
        a = self.alpha()
        if flat.is_cuda and _ext.available():
            if counters is not None:
                counters[1].fill_(self.iterations)
                _ext.ops().adam_step(flat, grad.contiguous(), self.m, self.v, self.beta_1, self.beta_2,
                                     self.learning_rate, self.epsilon, float(grad_scale), counters)
            else:
                _ext.ops().adam_step(flat, grad.contiguous(), self.m, self.v, self.beta_1, self.beta_2, a,
                                     self.epsilon, float(grad_scale))
        else:
            g = grad * grad_scale if grad_scale != 1.0 else grad
            self.m.add_((g - self.m) * (1 - self.beta_1))
            self.v.add_((g * g - self.v) * (1 - self.beta_2))
            flat.sub_(a * self.m / (self.v.sqrt() + self.epsilon))
        self.iterations += 1

    def state_dict(self) -> Dict[str, object]:
        return {"iterations": self.iterations, "m": None if self.m is None else self.m.detach().cpu(),
                "v": None if self.v is None else self.v.detach().cpu(), **self.get_config()}

    def load_state_dict(self, d, device=None) -> None:
        self.iterations = int(d["iterations"])
        if d.get("m") is not None:
            self.m = torch.as_tensor(d["m"]).float().to(device)
            self.v = torch.as_tensor(d["v"]).float().to(device)
