"""Deterministic HIP training (SURVEY §5 determinism; ``ops/train_ops.set_deterministic``).

In deterministic mode every reduction of the training step runs in a fixed order (BN moments, head
and dgrad sums: per-workgroup / per-sample partials + ``det_reduce_kernel``; weight gradients:
row-group partial slots), so
* two runs of the same steps give bitwise-identical weights, eagerly and as HIP-graph replays;
* a 2-rank data-parallel step (SyncBN + gradient all-reduce, ranks sharing the box's GPU over gloo)
  matches the 1-rank step to 1e-6 in gradient and BN statistics (only the cross-rank summation
  grouping differs)."""
import os

import numpy as np
import pytest
import torch

from .dist_utils import run_ranks

pytestmark = pytest.mark.gpu

_LAST = {}  # the last model _train built (its workspace holds the step's gradient)


def _data(n=256, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 60, 4, generator=g)
    y = (torch.rand(n, generator=g) > 0.6).float()
    return x, y


def _train(steps=3, graph="0"):
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D

    os.environ["APNEAUQ_TRAIN_GRAPH"] = graph
    x, y = _data()
    x, y = x.cuda(), y.cuda()
    m = AlarconCNN1D(seed=11, device="cuda")
    losses = [float(m.train_step(x[i * 64:(i + 1) * 64], y[i * 64:(i + 1) * 64])) for i in range(steps)]
    _LAST["model"] = m
    return losses, m.store.flat.clone(), m.store.stats.clone()


def _last_grad():
    m = _LAST["model"]
    ws = getattr(m, "_train_ws", None)
    return ws.grad.clone()


@pytest.fixture
def graph_env():
    old_graph = os.environ.get("APNEAUQ_TRAIN_GRAPH")
    yield
    if old_graph is None:
        os.environ.pop("APNEAUQ_TRAIN_GRAPH", None)
    else:
        os.environ["APNEAUQ_TRAIN_GRAPH"] = old_graph


def test_deterministic_training_is_bitwise_reproducible(deterministic, graph_env):
    l1, w1, s1 = _train(graph="0")
    l2, w2, s2 = _train(graph="0")
    assert l1 == l2
    assert torch.equal(w1, w2) and torch.equal(s1, s2)
    lg, wg, sg = _train(graph="1")  # the captured step replays the same kernels in the same order
    assert lg == l1
    assert torch.equal(wg, w1) and torch.equal(sg, s1)


def test_deterministic_mode_matches_atomic_mode(deterministic, graph_env):
    """One step from identical weights: the deterministic and the atomic mode differ only in the fp32
    summation order of the cross-workgroup sums (later steps are compared within one mode only)."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops

    ld, wd, _ = _train(steps=1, graph="0")
    gd = _last_grad()
    train_ops.set_deterministic(False)
    la, wa, _ = _train(steps=1, graph="0")
    ga = _last_grad()
    assert abs(ld[0] - la[0]) <= 1e-5 * abs(la[0])
    assert ((gd - ga).norm() / ga.norm()).item() < 1e-2



def _dp_step(rank, world):
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops
    from uncertaintyquantification_sleepapnea_1dcnn_amd.parallel.data_parallel import DPContext, split_batch

    train_ops.set_deterministic(True)
    x, y = _data(128, 5)
    m = AlarconCNN1D(seed=3, device="cuda")
    m.dp = DPContext(None, world, rank)
    idx, off = split_batch(torch.arange(x.shape[0]), m.dp)
    m.train_step(x[idx].cuda(), y[idx].cuda(), dp_step=(x.shape[0], off))
    return m.store.flat.cpu(), m.store.stats.cpu(), m._train_ws.grad.cpu()


def test_deterministic_dp_two_ranks_matches_one_rank(deterministic, graph_env):
    """The all-reduced gradient and the BN statistics of the 2-rank step match the 1-rank step to
    1e-6.  Weights after Adam: to 1e-6 except where a gradient cancels to ~epsilon (1e-7), where Adam's
    per-coordinate normalisation turns the fp32 summation-grouping residue into up to ~2 % of lr."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D

    os.environ["APNEAUQ_TRAIN_GRAPH"] = "0"
    res = run_ranks(_dp_step, 2, gpu=True)
    x, y = _data(128, 5)
    m = AlarconCNN1D(seed=3, device="cuda")
    m.train_step(x.cuda(), y.cuda())
    g1 = m._train_ws.grad.cpu()
    w1 = m.store.flat.cpu()
    for flat, stats, grad in res:
        torch.testing.assert_close(grad, g1, atol=1e-6, rtol=0)
        torch.testing.assert_close(stats, m.store.stats.cpu(), atol=1e-6, rtol=1e-6)
        d = (flat - w1).abs()
        assert d.max().item() < 2e-5 * m.optimizer.learning_rate / 1e-3
        assert (d > 1e-6).float().mean().item() < 1e-4, (d > 1e-6).sum().item()
    torch.testing.assert_close(res[0][0], res[1][0], atol=0, rtol=0)  # both ranks hold the same weights
