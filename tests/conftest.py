import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU on this machine")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def deterministic():
    """Deterministic HIP training (``ops/train_ops.set_deterministic``): every cross-workgroup sum of
    the reference-architecture and generic training kernels in a fixed order, so equivalent step
    sequences (eager / graph replay / member-batched / concurrent) give bitwise-identical results."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, train_ops

    _ext.require()
    old = train_ops.DETERMINISTIC
    train_ops.set_deterministic(True)
    yield
    train_ops.set_deterministic(old)
