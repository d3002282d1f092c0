"""GPU numerics of the UQ reduce / bootstrap / Adam HIP kernels vs fp32/fp64 host references."""
import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import uq as uq_ops
from uncertaintyquantification_sleepapnea_1dcnn_amd.training.optim import Adam
from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import metrics as M

pytestmark = pytest.mark.gpu


def test_uq_reduce_matches_numpy():
    _ext.require()
    rs = np.random.RandomState(0)
    p = np.clip(rs.rand(50, 3001), 0, 1).astype(np.float32)
    p[:, 0] = 0.0
    p[:, 1] = 1.0
    m = uq_ops.metrics(torch.from_numpy(p).cuda()).cpu().numpy()
    w = M.per_window(p)
    np.testing.assert_allclose(m[uq_ops.MEAN], w["mean_pred"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(m[uq_ops.VAR], w["pred_variance"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(m[uq_ops.ENT_NATS], w["total_pred_entropy"], rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(m[uq_ops.EXP_ENT], w["expected_aleatoric_entropy"], rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(m[uq_ops.MI], w["mutual_info"], rtol=1e-3, atol=5e-6)
    np.testing.assert_allclose(m[uq_ops.ENT_BITS], M.binary_entropy_bits(w["mean_pred"]), rtol=1e-4, atol=2e-6)
    np.testing.assert_array_equal(m[uq_ops.LABEL], (w["mean_pred"] > 0.5).astype(np.float32))


@pytest.mark.parametrize("parity", [True, False])
def test_bootstrap_kernel(parity):
    _ext.require()
    rs = np.random.RandomState(1)
    p = rs.rand(7, 2000).astype(np.float32)
    y = (rs.rand(2000) > 0.7).astype(np.int32)
    w = M.per_window(p)
    mt = uq_ops.metrics(torch.from_numpy(p).cuda())
    if parity:
        idx = M.parity_bootstrap_indices(2000, 20, 2025)
        got = uq_ops.bootstrap(mt, torch.from_numpy(y).cuda(), 20, idx=torch.from_numpy(idx.astype(np.int32)).cuda())
    else:
        idx = uq_ops._hash_idx(2000, 20, 2025, "cpu").numpy()
        got = uq_ops.bootstrap(mt, torch.from_numpy(y).cuda(), 20, seed=2025)
    ref = M.bootstrap_from_windows(w, y, idx)
    got = got.cpu().numpy()
    for b in range(20):
        np.testing.assert_allclose(got[b], [ref[b][k] for k in M.AGG_KEYS], rtol=2e-4, atol=1e-7)


@pytest.mark.parametrize("parity", [True, False])
def test_bootstrap_partial_kernel_matches_eager(parity):
    """Sharded bootstrap kernel: per-shard (B, 8) sums equal the eager sums, and the
    summed shards finalize to the single-launch bootstrap."""
    _ext.require()
    rs = np.random.RandomState(2)
    n, B = 3001, 16
    p = torch.from_numpy(rs.rand(5, n).astype(np.float32)).cuda()
    y = torch.from_numpy((rs.rand(n) > 0.6).astype(np.int32)).cuda()
    mt = uq_ops.metrics(p)
    idx = torch.from_numpy(M.parity_bootstrap_indices(n, B, 7).astype(np.int32)).cuda() if parity else None
    tot = torch.zeros(B, 8, dtype=torch.float64, device="cuda")
    for s, e in ((0, 1000), (1000, 1001), (1001, n)):
        part = uq_ops.bootstrap_partial(mt[:, s:e].contiguous(), y[s:e], B, n, s, idx=idx, seed=7)
        ref = uq_ops.bootstrap_partial_eager(mt[:, s:e].cpu(), y[s:e].cpu(), None if idx is None else idx.cpu(), 7, B, n, s)
        torch.testing.assert_close(part.cpu(), ref, rtol=1e-9, atol=1e-9)
        tot += part
    full = uq_ops.bootstrap(mt, y, B, idx=idx, seed=7)
    torch.testing.assert_close(uq_ops.finalize_bootstrap_sums(tot, n), full, rtol=1e-12, atol=1e-12)


def test_adam_kernel_matches_eager():
    _ext.require()
    n = 851457
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) for _ in range(3)]
    a, b = Adam(1e-3), Adam(1e-3)
    pa, pb = p0.clone(), p0.clone().cuda()
    for gr in grads:
        a.step(pa, gr)
        b.step(pb, gr.cuda())
    torch.testing.assert_close(pb.cpu(), pa, rtol=1e-6, atol=1e-6)


def test_metrics_kernel_matches_bucketize():
    """K10 (csrc/metrics.hip): device accuracy / AUC counters == the host bucketize path, including
    predictions exactly on thresholds, and no host sync per batch."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.training import metrics as TM

    _ext.require()
    g = torch.Generator().manual_seed(0)
    thr = torch.tensor(TM.keras_thresholds(), dtype=torch.float32)
    p = torch.cat([torch.rand(5000, generator=g), thr[1:-1], torch.tensor([0.0, 1.0, 0.5])])
    y = (torch.rand(p.numel(), generator=g) > 0.6).float()
    acc_d, auc_d, acc_h, auc_h = TM.BinaryAccuracy(), TM.AUC(), TM.BinaryAccuracy(), TM.AUC()
    for s in range(0, p.numel(), 1024):
        acc_d.update_state(y[s: s + 1024].cuda(), p[s: s + 1024].cuda())
        auc_d.update_state(y[s: s + 1024].cuda(), p[s: s + 1024].cuda())
        acc_h.update_state(y[s: s + 1024], p[s: s + 1024])
        auc_h.update_state(y[s: s + 1024], p[s: s + 1024])
    assert auc_d._counts is not None and acc_d._counts is not None  # accumulated on the device
    np.testing.assert_array_equal(auc_d.confusion()[0], auc_h.confusion()[0])
    np.testing.assert_array_equal(auc_d.pos_hist, auc_h.pos_hist)
    np.testing.assert_array_equal(auc_d.neg_hist, auc_h.neg_hist)
    assert acc_d.result() == acc_h.result()
    assert abs(auc_d.result() - auc_h.result()) < 1e-12


def test_zero_buffers_one_launch():
    """ops zero_buffers: several buffers of mixed dtypes / sizes (not multiples of 16 B, unaligned
    views) cleared by one launch; neighbouring memory untouched."""
    import torch

    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext

    _ext.require()
    dev = torch.device("cuda")
    a = torch.full((1001,), 3.0, dtype=torch.float64, device=dev)
    b = torch.full((7,), 2.0, device=dev)
    big = torch.full((1 << 20,), 1.0, device=dev)
    c = big[1: 1 + 777777]  # 4-B aligned, not 16-B aligned
    _ext.ops().zero_buffers([a, b, c])
    torch.cuda.synchronize()
    assert a.abs().sum().item() == 0 and b.abs().sum().item() == 0 and c.abs().sum().item() == 0
    assert big[0].item() == 1.0 and big[1 + 777777:].eq(1.0).all().item()
