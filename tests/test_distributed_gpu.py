"""Sharded UQ on the HIP paths: 2 ranks share the box's GPU over gloo (RCCL needs a GPU per rank;
the 8-GPU RCCL path is the driver's scaling bench).  Checks the fused running-BN path and the
layer-wise batch-BN path with SyncBN against a single-process run."""
import numpy as np
import pytest
import torch

from .dist_utils import run_ranks

pytestmark = pytest.mark.gpu


def _x():
    return torch.randn(203, 60, 4, generator=torch.Generator().manual_seed(8))


def _uq(rank, world, bn_mode):
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

    m = AlarconCNN1D(seed=4, device="cuda")
    mcd = U.mc_dropout_predict(m, _x(), n_pred=4, bn_mode=bn_mode)
    de = U.deep_ensembles_predict([AlarconCNN1D(seed=10 + i, device="cuda") for i in range(3)], _x())
    return mcd, de, m.store.stats.cpu()


@pytest.mark.parametrize("bn_mode", ["running", "batch"])
def test_sharded_uq_hip_matches_single_process(bn_mode):
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

    res = run_ranks(_uq, 2, (bn_mode,), gpu=True)
    m = AlarconCNN1D(seed=4, device="cuda")
    mcd = U.mc_dropout_predict(m, _x(), n_pred=4, bn_mode=bn_mode, distributed=False)
    de = U.deep_ensembles_predict([AlarconCNN1D(seed=10 + i, device="cuda") for i in range(3)], _x(), distributed=False)
    for r_mcd, r_de, r_stats in res:
        if bn_mode == "running":  # fused kernel: masks keyed by global window id -> bitwise equal
            np.testing.assert_array_equal(r_mcd, mcd)
        else:  # SyncBN: same statistics up to summation order (bf16 activations)
            np.testing.assert_allclose(r_mcd, mcd, atol=2e-2, rtol=2e-2)
            torch.testing.assert_close(r_stats, m.store.stats.cpu(), atol=2e-3, rtol=2e-2)
        np.testing.assert_array_equal(r_de, de)
