"""GPU numerics of the fp32 precision path (``csrc/gf32_conv.hip`` + the fp32 instantiations of the
generic BN / pool / dropout / head kernels, ``ops/generic_train.py``): the reference trains and infers in
fp32 (Keras defaults: ``/root/reference/models/cnn_baseline_train.py:100-102,210-217``,
``uncertainty_quantification/uq_techniques.py:22-30``), so

* ``train_precision="fp32"`` training steps of every architecture (the reference CNN included) give
  per-tensor gradients within 1e-4 of fp32 autograd over the reference ops, and 10-epoch loss histories
  within 1e-3 of the PyTorch fp32 backend;
* ``precision="fp32"`` inference of the non-reference architectures (the pooled ``ensemble_cnn`` members of
  ``evaluate_de_global.py:18-38``, the 30 s single-channel window) -- Deep-Ensemble predict, standard and
  batch-BN MC Dropout -- is within 1e-5 |dp| of the fp32 reference;
* the fp32 step is deterministic: its graph replay equals the eager step bitwise."""
import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import _ext, generic_train
from uncertaintyquantification_sleepapnea_1dcnn_amd.training import step as tstep

from .test_generic_gpu import SPECS
from .test_train_gpu import TRAIN_PASS_BASE

pytestmark = pytest.mark.gpu

ALL = dict(SPECS, reference=DEFAULT_SPEC)


def _batch(spec, n, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, spec.input_length, spec.input_channels, generator=g)
    y = (torch.rand(n, generator=g) > 0.5).float()
    return x.cuda(), y.cuda()


def _grads64(model, x, y):
    """float64 CPU autograd over the reference ops: the exact oracle (GPU fp32 autograd is itself only
    fp32-accurate -- its MIOpen convolutions may use reduced-precision paths -- so it cannot pin 1e-4)."""
    store = model.store
    flat = store.flat.detach().cpu().double().requires_grad_(True)
    stats = store.stats.detach().cpu().double()
    p = {}
    for n in store.trainable:
        off = store.offsets[n]
        p[n] = flat[off: off + store.views[n].numel()].view(store.shapes[n])
    off = 0
    for n in store.nontrainable:
        k = store.views[n].numel()
        p[n] = stats[off: off + k].view(store.shapes[n])
        off += k
    xc, yc = x.detach().cpu().double(), y.detach().cpu().double()
    logits = R.forward(model.spec, p, xc, dropout=True, bn_batch_stats=True, update_moving=True, seed=model.seed,
                       pass_id=TRAIN_PASS_BASE + model._train_step_counter, sample_ids=torch.arange(xc.shape[0]),
                       return_logits=True, dtype=torch.float64)
    lv = torch.nn.functional.binary_cross_entropy_with_logits(logits.reshape(-1), yc, reduction="none")
    lv.mean().backward()
    dev = store.flat.device
    return lv.sum().item(), flat.grad.detach().float().to(dev), stats.float().to(dev)


@pytest.mark.parametrize("name", list(ALL))
def test_fp32_train_step_matches_autograd(name):
    _ext.require()
    spec = ALL[name]
    m = AlarconCNN1D(spec=spec, seed=5, device="cuda", train_precision="fp32")
    assert tstep._backend(m) == "hip_generic"
    x, y = _batch(spec, 64, 3)
    m.optimizer.learning_rate = 0.0
    ref_loss, ref_grad, ref_stats = _grads64(m, x, y)
    loss, _ = generic_train.train_step(m, x, y)
    ws = m._gtrain_ws32
    assert ws.f32 and ws.z[0].dtype == torch.float32
    assert abs(loss.item() - ref_loss) <= 1e-5 * ref_loss
    st = m.store
    bad = []
    for nm in st.trainable:
        off, k = st.offsets[nm], st.views[nm].numel()
        hip, ref = ws.grad[off: off + k], ref_grad[off: off + k]
        err = (hip - ref).norm().item()
        # conv biases feed a batch-statistics BN: their true gradient is a cancellation residual of size
        # ~fp32 rounding, so they are held to an absolute bound
        if err > 1e-4 * ref.norm().item() and err > 1e-6:
            bad.append((nm, err, ref.norm().item()))
    assert not bad, bad
    torch.testing.assert_close(st.stats, ref_stats, atol=1e-6, rtol=1e-5)


def test_fp32_graph_step_is_the_eager_step(monkeypatch):
    _ext.require()
    spec = SPECS["pooled"]
    x, y = _batch(spec, 256, 7)
    runs = []
    for graph in ("0", "1"):
        monkeypatch.setenv("APNEAUQ_TRAIN_GRAPH", graph)
        m = AlarconCNN1D(spec=spec, seed=4, device="cuda", train_precision="fp32")
        losses = [float(m.train_step(x[i * 64:(i + 1) * 64], y[i * 64:(i + 1) * 64])) for i in range(4)]
        runs.append((losses, m.store.flat.clone(), m.store.stats.clone()))
        if graph == "1":
            assert 64 in m._gtrain_graphs and m._gtrain_graphs[64].f32
    (le, we, se), (lg, wg, sg) = runs
    assert lg == le
    assert torch.equal(wg, we) and torch.equal(sg, se)


def test_fp32_training_loss_history_matches_torch_backend(monkeypatch):
    """10 epochs of Keras fit (batch 1024, validation_split 0.1) on the HIP fp32 kernels and on fp32
    autograd from the same init, data and dropout masks: every epoch's loss within 1e-3 relative, no
    absolute floor.  The windows are the synthetic apnea set with extra noise, re-standardised per
    window (as tests/test_train_gpu.py's bf16 parity test), so the task does not saturate: every
    epoch's loss stays >= 0.05 and is decided by the whole set, not by a handful of windows."""
    _ext.require()
    # the torch side in true fp32 (no TF32-style reduced-precision convolutions / matmuls)
    monkeypatch.setattr(torch.backends.cudnn, "allow_tf32", False)
    monkeypatch.setattr(torch.backends.cuda.matmul, "allow_tf32", False)
    from uncertaintyquantification_sleepapnea_1dcnn_amd.data.synthetic import synthetic_windows

    x, y, _ = synthetic_windows(8192, seed=17)
    rs = np.random.RandomState(17)
    x = (x + rs.randn(*x.shape).astype(np.float32) * 1.6).astype(np.float32)
    x = ((x - x.mean(1, keepdims=True)) / (x.std(1, keepdims=True) + 1e-8)).astype(np.float32)
    hist = {}
    for backend in ("auto", "torch"):
        monkeypatch.setenv("APNEAUQ_TRAIN_BACKEND", backend)
        m = AlarconCNN1D(seed=2025, device="cuda", train_precision="fp32")
        hist[backend] = m.fit(x, y.astype(np.float32), batch_size=1024, epochs=10, validation_split=0.1,
                              verbose=0).history["loss"]
    assert len(hist["auto"]) == 10 and min(hist["auto"]) >= 0.05, hist["auto"]
    np.testing.assert_allclose(hist["auto"], hist["torch"], rtol=1e-3, atol=0)


@pytest.mark.parametrize("name", ["pooled", "single30"])
def test_fp32_inference_matches_reference(name):
    """Deep-Ensemble predict (members' moving statistics), standard MC Dropout and the reference's
    batch-BN MC Dropout of non-reference architectures at fp32 (precision defaults to "fp32")."""
    _ext.require()
    from uncertaintyquantification_sleepapnea_1dcnn_amd.uq import uq_techniques as U

    spec = SPECS[name]
    ps = [R.synthetic_params(spec, 40 + i) for i in range(3)]
    models = [AlarconCNN1D(spec=spec, seed=40 + i, device="cuda", params=p) for i, p in enumerate(ps)]
    assert all(m.precision == "fp32" and not m.uses_x3() for m in models)
    x = torch.randn(75, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(2))
    de = U.deep_ensembles_predict(models, x.numpy())
    for i, p in enumerate(ps):
        ref = R.forward(spec, p, x).reshape(-1).numpy()
        assert np.abs(de[i, :, 0] - ref).max() <= 1e-5
    m0, T = models[0], 3
    run = U.mc_dropout_predict(m0, x.numpy(), n_pred=T, bn_mode="running", seed=9)
    for t in range(T):
        ref = R.forward(spec, ps[0], x, dropout=True, seed=9, pass_id=t, sample_ids=torch.arange(75)).reshape(-1)
        assert np.abs(run[t, :, 0] - ref.numpy()).max() <= 1e-5
    mb = AlarconCNN1D(spec=spec, seed=41, device="cuda", params=ps[1])
    pc = {k: v.clone() for k, v in ps[1].items()}
    bat = U.mc_dropout_predict(mb, x.numpy(), n_pred=T, bn_mode="batch", seed=5)
    for t in range(T):
        ref = R.forward(spec, pc, x, dropout=True, bn_batch_stats=True, update_moving=True, seed=5, pass_id=t,
                        sample_ids=torch.arange(75)).reshape(-1)
        assert np.abs(bat[t, :, 0] - ref.numpy()).max() <= 1e-5, t
    for k, v in pc.items():  # the moving-average side effect of model(x, training=True), per pass
        torch.testing.assert_close(mb.store.as_dict()[k].cpu(), v, atol=1e-6, rtol=1e-5)


def test_fp32_inference_window_chunks_match_one_chunk(monkeypatch):
    """fp32 inference of a non-reference architecture runs in bounded window chunks (the
    cached workspace stays bounded); the dropout keys stay global, so 7-window chunks give the same
    standard-MC-Dropout probabilities as one chunk."""
    _ext.require()
    spec = SPECS["pooled"]
    m = AlarconCNN1D(spec=spec, seed=3, device="cuda", params=R.synthetic_params(spec, 3))
    x = torch.randn(40, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(4)).cuda()
    one = generic_train.forward_running_f32(m, x, n_pass=3, dropout=True, seed=11, window_offset=5)
    per = sum((L + b.kernel_size) * c + L * c2 for L, b, c, c2 in
              zip(spec.lengths(), spec.blocks, spec.channels(), spec.channels()[1:])) * 4
    monkeypatch.setattr(generic_train, "F32_INFER_WS_BYTES", 7 * per)
    assert generic_train._f32_chunk_windows(m) == 7
    m._gfwd_ws32 = None
    chunked = generic_train.forward_running_f32(m, x, n_pass=3, dropout=True, seed=11, window_offset=5)
    torch.testing.assert_close(chunked, one, atol=0, rtol=0)
    assert m._gfwd_ws32.B < 40
