"""Layer-wise HIP training kernels (conv fwd/dgrad/wgrad with fused BN/dropout).  Placeholder
until the kernels land: ``supports`` returns False so training uses the autograd path."""
from __future__ import annotations


def supports(spec) -> bool:
    return False


def train_step(model, x, y, grad_allreduce=None):  # pragma: no cover
    raise NotImplementedError
