"""Keras-semantics tests (SURVEY §4 test 3): tail validation split, EarlyStopping restore rule,
BN momentum/epsilon, Adam epsilon, AUC thresholds, loss reduction on a learnable task."""
import numpy as np
import pytest
import torch
from sklearn.metrics import roc_auc_score

from uncertaintyquantification_sleepapnea_1dcnn_amd.data.synthetic import synthetic_windows
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.training.callbacks import EarlyStopping
from uncertaintyquantification_sleepapnea_1dcnn_amd.training.metrics import AUC, keras_thresholds
from uncertaintyquantification_sleepapnea_1dcnn_amd.training.optim import Adam


class _Dummy:
    def __init__(self):
        self.w = 0
        self.stop_training = False
        self.restored = None

    def snapshot(self):
        return self.w

    def restore(self, s):
        self.restored = s


def test_early_stopping_keras_rule():
    es = EarlyStopping(patience=2, restore_best_weights=True)
    m = _Dummy()
    es.set_model(m)
    es.on_train_begin()
    for epoch, vl in enumerate([1.0, 0.8, 0.9, 0.95, 0.7]):
        m.w = epoch
        es.on_epoch_end(epoch, {"val_loss": vl})
        if m.stop_training:
            break
    assert m.stop_training and es.stopped_epoch == 3 and m.restored == 1  # best epoch 1 restored at the stop
    # no restore when training ends naturally
    es2 = EarlyStopping(patience=5, restore_best_weights=True)
    m2 = _Dummy()
    es2.set_model(m2)
    es2.on_train_begin()
    for epoch, vl in enumerate([1.0, 0.8, 0.9]):
        es2.on_epoch_end(epoch, {"val_loss": vl})
    assert not m2.stop_training and m2.restored is None


def test_adam_keras_formula():
    p = torch.tensor([1.0, -2.0])
    g = torch.tensor([0.5, 0.25])
    opt = Adam(1e-3)
    opt.step(p, g)
    # first step: m = 0.1 g, v = 0.001 g^2, alpha = lr*sqrt(1-0.999)/(1-0.9)
    alpha = 1e-3 * np.sqrt(1 - 0.999) / (1 - 0.9)
    m, v = 0.1 * g, 0.001 * g * g
    exp = torch.tensor([1.0, -2.0]) - alpha * m / (v.sqrt() + 1e-7)
    torch.testing.assert_close(p, exp)


def test_auc_matches_threshold_rule():
    rs = np.random.RandomState(0)
    y = (rs.rand(2000) > 0.5).astype(np.float32)
    p = np.clip(y * 0.3 + rs.rand(2000) * 0.7, 0, 1).astype(np.float32)
    a = AUC()
    a.update_state(torch.from_numpy(y[:700]), torch.from_numpy(p[:700]))
    a.update_state(torch.from_numpy(y[700:]), torch.from_numpy(p[700:]))
    thr = keras_thresholds()
    tp = np.array([((p > t) & (y == 1)).sum() for t in thr])
    fp = np.array([((p > t) & (y == 0)).sum() for t in thr])
    tpr, fpr = tp / (y == 1).sum(), fp / (y == 0).sum()
    ref = np.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2)
    assert a.result() == pytest.approx(ref, abs=1e-9)
    assert a.result() == pytest.approx(roc_auc_score(y, p), abs=5e-3)


def test_bn_moving_update_and_tail_validation_split():
    m = AlarconCNN1D(seed=0, device="cpu")
    x, y, _ = synthetic_windows(100, seed=0)
    before = m.store.views["batchnorm_1/moving_mean"].clone()
    m(torch.from_numpy(x), training=True)
    after = m.store.views["batchnorm_1/moving_mean"]
    h = torch.relu(torch.nn.functional.conv1d(torch.nn.functional.pad(torch.from_numpy(x).transpose(1, 2), (3, 3)),
                                              m.store.views["conv1d_1/kernel"].permute(2, 1, 0),
                                              m.store.views["conv1d_1/bias"]))
    torch.testing.assert_close(after, before * 0.99 + h.mean((0, 2)) * 0.01, atol=1e-6, rtol=1e-5)
    # tail split: the validation set is the LAST 10 % of the arrays (not shuffled)
    seen = {}

    def spy(model, X, Y, bs=1024):
        seen["val"] = X.clone()
        return 0.5, 0.5, 0.5

    import uncertaintyquantification_sleepapnea_1dcnn_amd.training.trainer as T

    orig = T.evaluate_arrays
    T.evaluate_arrays = spy
    try:
        m.fit(x, y.astype(np.float32), batch_size=32, epochs=1, validation_split=0.1, verbose=0)
    finally:
        T.evaluate_arrays = orig
    torch.testing.assert_close(seen["val"], torch.from_numpy(x[90:]))


def test_training_learns_cpu():
    x, y, _ = synthetic_windows(512, seed=3)
    m = AlarconCNN1D(seed=3, device="cpu")
    h = m.fit(x, y.astype(np.float32), batch_size=64, epochs=2, validation_split=0.1, verbose=0)
    assert h.history["loss"][1] < h.history["loss"][0]


@pytest.mark.parametrize("pooled", [False, True])
def test_generic_train_emulation_matches_autograd(pooled, monkeypatch):
    """The bf16-dataflow oracle of the generic HIP training path (tests/generic_train_emulation.py)
    is exact fp32 backprop once its quantisation points are switched off (pool routing, dropout,
    BN backward, dgrad/wgrad index algebra)."""
    import dataclasses

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import BlockSpec, ModelSpec

    from . import generic_train_emulation as E

    monkeypatch.setattr(E, "bf", lambda t: t.float())
    spec = ModelSpec(31, 3, tuple(BlockSpec(f, k, r, pooled and i != 1) for i, (f, k, r) in
                                  enumerate([(8, 5, 0.3), (12, 3, 0.2), (16, 1, 0.5)])))
    p = R.synthetic_params(spec, 3)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(9, 31, 3, generator=g)
    y = (torch.rand(9, generator=g) > 0.5).float()
    loss, _, eg, _ = E.emulate_generic_step(spec, p, x, y, seed=4, pass_id=7)
    q = {k: (v.clone().requires_grad_(True) if not k.endswith(("moving_mean", "moving_variance")) else v.clone())
         for k, v in p.items()}
    lg = R.forward(spec, q, x, dropout=True, bn_batch_stats=True, seed=4, pass_id=7, return_logits=True)
    lv = torch.nn.functional.binary_cross_entropy_with_logits(lg.reshape(-1), y, reduction="none")
    lv.mean().backward()
    assert abs(lv.sum().item() - loss) < 1e-4 * max(1.0, loss)
    for k, v in eg.items():
        torch.testing.assert_close(v.reshape(q[k].grad.shape), q[k].grad, atol=1e-5, rtol=1e-4)


def test_fit_concurrent_equals_sequential_fit():
    """Members stepped round-robin (training/trainer.py:fit_concurrent) train exactly like
    back-to-back fit() calls: same histories and bitwise-equal weights (CPU, no streams)."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.training.trainer import fit_concurrent

    g = torch.Generator().manual_seed(1)
    x = torch.randn(96, 60, 4, generator=g)
    y = (x[:, :, 0].mean(1) > 0).float()
    kw = dict(epochs=2, batch_size=32, validation_split=0.25, verbose=0)
    seq = [AlarconCNN1D(seed=10 + i, device="cpu") for i in range(3)]
    h_seq = [m.fit(x, y, callbacks=[EarlyStopping(patience=1)], **kw) for m in seq]
    con = [AlarconCNN1D(seed=10 + i, device="cpu") for i in range(3)]
    h_con = fit_concurrent(con, x, y, callbacks=[[EarlyStopping(patience=1)] for _ in con], **kw)
    for a, b, hs, hc in zip(seq, con, h_seq, h_con):
        assert hs.history == hc.history
        for wa, wb in zip(a.get_weights(), b.get_weights()):
            np.testing.assert_array_equal(wa, wb)


def test_graph_bound_key_tracks_optimizer_scalars():
    """A captured training graph is re-captured when lr / betas / epsilon change."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import train_ops

    m = AlarconCNN1D(seed=1, device="cpu")
    k1 = train_ops.bound_key(m)
    assert train_ops._same_bound(k1, train_ops.bound_key(m))
    m.optimizer.learning_rate = 5e-4
    assert not train_ops._same_bound(k1, train_ops.bound_key(m))


def test_fused_input_copy_only_takes_matching_device_batches():
    """the graphed step's fused input copy (ops/train_ops.py ``_inputs_direct``) reads the batch
    in place, so it applies only to fp32 contiguous (n, 60, C_in) windows and (n,) labels on the
    workspace's own device; a CPU batch, a wrong channel count or shape falls back to ``copy_``."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops.train_ops import _inputs_direct

    dev = torch.device("cpu")
    x, y = torch.zeros(8, 60, 4), torch.zeros(8)
    assert not _inputs_direct([x], [y], 8, dev, 4)  # CPU tensors are never read by the kernel
    meta = torch.device("meta")
    xm, ym = torch.zeros(8, 60, 4, device=meta), torch.zeros(8, device=meta)
    assert not _inputs_direct([xm], [ym], 8, dev, 4)  # not a GPU tensor
    assert not _inputs_direct([x[:, :, :3].contiguous()], [y], 8, dev, 4)
    assert not _inputs_direct([x], [y[:7]], 8, dev, 4)
    assert not _inputs_direct([x.double()], [y], 8, dev, 4)


def test_wgrad_partial_buffer_covers_every_smaller_batch():
    """csrc/train_conv.hip train_wgrad_part_floats: a workspace of capacity B serves every batch n <= B
    (a partial last batch runs its own row grouping, which is not monotone in n: the row-tile cap changes
    at 2048 samples), so the size is the running maximum -- non-decreasing in B -- and holds the fused
    step's wgrad<0> region behind the shared one.  Host-only op: runs wherever the extension loads."""
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext

    if not _ext.load():
        pytest.skip("HIP extension not built")
    o = _ext.ops()
    sizes = [o.train_wgrad_part_size(b) for b in list(range(1, 80)) + list(range(2000, 2100)) + [4096, 8192]]
    assert all(b >= a for a, b in zip(sizes, sizes[1:]))
    assert o.train_wgrad_part_size(2050) >= o.train_wgrad_part_size(2048) > 0
