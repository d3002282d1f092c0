"""CPU tier: architecture spec, Keras-default init, 38-array checkpoint layout, counter-based
dropout masks (NumPy == torch, rate), fused-blob packing (bf16 emulation == fp32 reference)."""
import numpy as np
import pytest
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.cnn import AlarconCNN1D, load_model
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC, ModelSpec
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused, rng


def test_spec_counts():
    assert DEFAULT_SPEC.num_params() == (853441, 851457)
    assert DEFAULT_SPEC.forward_macs() == 50903136
    assert len(DEFAULT_SPEC.weight_names()) == 38
    assert DEFAULT_SPEC.weight_shapes()[0] == (7, 4, 128)
    assert DEFAULT_SPEC.weight_shapes()[-2:] == [(96, 1), (1,)]
    s = ModelSpec.from_dict(DEFAULT_SPEC.to_dict())
    assert s == DEFAULT_SPEC


def test_keras_init():
    p = R.init_params(DEFAULT_SPEC, 0)
    k = p["conv1d_2/kernel"]
    lim = np.sqrt(6.0 / (5 * 128 + 5 * 192))
    assert float(k.abs().max()) <= lim + 1e-6 and float(k.abs().max()) > 0.9 * lim
    assert torch.all(p["batchnorm_3/moving_variance"] == 1) and torch.all(p["conv1d_3/bias"] == 0)


def test_checkpoint_roundtrip(tmp_path):
    m = AlarconCNN1D(seed=1, device="cpu")
    w = m.get_weights()
    assert len(w) == 38 and [a.shape for a in w] == [tuple(s) for s in DEFAULT_SPEC.weight_shapes()]
    w[5] = w[5] + 0.5  # moving variance of BN1
    m.set_weights(w)
    path = m.save(str(tmp_path / "AlCNN_smote_seed21.keras"))
    m2 = load_model(path, device="cpu")
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)
    # a .keras path is a genuine Keras v3 archive (utils/keras_io.py); other names are .npz
    import zipfile

    with zipfile.ZipFile(path) as z:
        assert {"config.json", "model.weights.h5"} <= set(z.namelist())
    npz = m.save(str(tmp_path / "w.npz"))
    with np.load(npz, allow_pickle=False) as z:
        assert "conv1d_1/kernel" in z.files and "output_layer/bias" in z.files


def test_dropout_masks_numpy_equals_torch_and_rate():
    key = rng.stream_key(2025, 3, 17)
    samples = np.arange(100, 140)
    a = rng.keep_mask_np(key, samples, 60, 96, 0.2)
    b = rng.keep_mask_torch(key, torch.from_numpy(samples), 60, 96, 0.2).numpy()
    np.testing.assert_array_equal(a, b)
    assert abs(a.mean() - 0.8) < 0.01
    c = rng.keep_mask_np(rng.stream_key(2025, 3, 18), samples, 60, 96, 0.2)
    assert (a != c).mean() > 0.2  # different pass -> different mask


def test_reference_forward_modes():
    m = AlarconCNN1D(seed=2, device="cpu")
    x = torch.randn(5, 60, 4)
    p1 = m(x)
    p2 = m(x)
    torch.testing.assert_close(p1, p2)  # inference is deterministic
    t1 = m(x, training=True)
    t2 = m(x, training=True)
    assert (t1 - t2).abs().max() > 0  # fresh dropout stream per call
    assert p1.shape == (5, 1) and torch.all((p1 > 0) & (p1 < 1))


def test_fused_packing_roundtrip_and_emulation():
    p = R.init_params(DEFAULT_SPEC, 3)
    for i in range(1, 7):
        c = DEFAULT_SPEC.blocks[i - 1].filters
        p[f"batchnorm_{i}/moving_mean"] = torch.rand(c) * 0.3
        p[f"batchnorm_{i}/moving_variance"] = torch.rand(c) + 0.5
    for i, b in enumerate(DEFAULT_SPEC.blocks, start=1):
        w = p[f"conv1d_{i}/kernel"]
        fr = fused.pack_conv_fragments(w)
        back = fused.unpack_conv_fragments(fr, *w.shape)
        torch.testing.assert_close(back, w.to(torch.bfloat16).float())
    blob = fused.pack_blob(DEFAULT_SPEC, p)
    assert blob.numel() == fused.layout()["bytes"]
    x = torch.randn(7, 60, 4)
    ref = R.forward(DEFAULT_SPEC, p, x, dropout=False, bn_batch_stats=False, return_logits=True).reshape(-1)
    emu = fused.emulate_blob_forward(blob, x, logits=True)
    assert (ref - emu).abs().max() < 0.05


def test_eager_comparator_matches_reference_forward():
    """bench/comparator.py's torch.nn model computes the same function as models/reference.py."""
    from bench.comparator import EagerCNN

    p = R.synthetic_params(DEFAULT_SPEC, 3)
    m = EagerCNN().load_keras(p).eval()
    x = torch.randn(16, 60, 4)
    with torch.no_grad():
        np.testing.assert_allclose(m(x).numpy(), R.forward(DEFAULT_SPEC, p, x).numpy(), rtol=1e-4, atol=1e-5)
        m.train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        ref = R.forward(DEFAULT_SPEC, p, x, training=True, dropout=False)
        np.testing.assert_allclose(m(x).numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)


def test_evaluate_classification_model_keys():
    from uncertaintyquantification_sleepapnea_1dcnn_amd.evaluation.evaluate_classification import (
        evaluate_classification_model)

    m = AlarconCNN1D(seed=1, device="cpu")
    x = torch.randn(64, 60, 4).numpy()
    y = (np.arange(64) % 3 == 0).astype(int)
    r = evaluate_classification_model(m, x, y, "t")
    assert len(r) == 14 and {"roc_auc", "auc_pr", "overall_sensitivity", "overall_specificity", "cohen_kappa", "mcc"} <= set(r)


def test_generic_emulation_matches_reference_pooled():
    """The bf16 emulation of the generic HIP path (ops/generic.py) against the fp32 reference for a
    pooled architecture and the 30 s single-channel shape, dropout on and off."""
    import dataclasses

    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import BlockSpec, ModelSpec
    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import generic

    pooled = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                            for i, b in enumerate(DEFAULT_SPEC.blocks)))
    single = ModelSpec(30, 1, (BlockSpec(32, 7, 0.3, True), BlockSpec(20, 3, 0.5, False)))
    assert generic.supports(pooled) and generic.supports(single)
    assert not generic.supports(ModelSpec.with_input((60, 4), pool=True))  # 6 pools: length 0
    for spec in (pooled, single):
        p = R.synthetic_params(spec, 4)
        x = torch.randn(9, spec.input_length, spec.input_channels, generator=torch.Generator().manual_seed(0))
        for drop in (False, True):
            a = generic.emulate(spec, p, x, dropout=drop, seed=3, pass_id=1)
            b = R.forward(spec, p, x, dropout=drop, bn_batch_stats=False, seed=3, pass_id=1)
            np.testing.assert_allclose(a.numpy(), b.numpy().reshape(-1), atol=3e-2)


def test_fused_pooled_dispatch_and_blob():
    """The pooled reference CNN (MaxPool1D after blocks 1-5) is the architecture of
    csrc/fused_tiled.hip (with the 30 s single-channel window): same parameter blob as the no-pool
    kernel; other pool patterns are not."""
    import dataclasses

    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused, generic

    pooled = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                            for i, b in enumerate(DEFAULT_SPEC.blocks)))
    two = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 2))
                                                         for i, b in enumerate(DEFAULT_SPEC.blocks)))
    from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import ModelSpec

    assert fused.pooled_supported(pooled) and not fused.supports(pooled)
    single = ModelSpec(30, 1, DEFAULT_SPEC.blocks)
    assert fused.tiled_net(pooled) == 0 and fused.tiled_net(single) == 1 and fused.tiled_net(DEFAULT_SPEC) is None
    assert fused.pack_blob(single, R.synthetic_params(single, 1)).numel() == fused.layout()["bytes"]
    assert not fused.pooled_supported(DEFAULT_SPEC) and not fused.pooled_supported(two)
    p = R.synthetic_params(pooled, 2)
    blob = fused.pack_blob(pooled, p)
    assert blob.numel() == fused.layout()["bytes"]
    pk = generic.pack(pooled, p)
    assert torch.equal(pk["tiled_blob"][0], blob)
    assert "tiled_blob" not in generic.pack(two, R.synthetic_params(two, 2))
    # the last block feeds the head in fp32 on the fused path: the emulation follows it
    x = torch.randn(5, 60, 4, generator=torch.Generator().manual_seed(1))
    a = generic.emulate(pooled, p, x, logits=True)
    b = generic.emulate(pooled, p, x, logits=True, last_fp32=True)
    assert torch.equal(a, b)


def test_fused_x3_blob_packing():
    """fp16x3 blob of the fp32 fused kernel (ops/fused.py:pack_blob_x3): the hi + lo fragments of each
    layer reproduce W within 2^-21 of max |W| (one power-of-two prescale per layer), the epilogue scale
    carries the inverse power of two, the layout matches the kernel's constants (fused_blob.h)."""
    import dataclasses

    from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import fused

    pooled = dataclasses.replace(DEFAULT_SPEC, blocks=tuple(dataclasses.replace(b, pool=(i < 5))
                                                            for i, b in enumerate(DEFAULT_SPEC.blocks)))
    p = R.synthetic_params(pooled, 3)
    blob = fused.pack_blob_x3(pooled, p)
    lay = fused.layout_x3()
    assert blob.numel() == lay["bytes"]
    ch, ks = fused.FUSED_CHANNELS, fused.FUSED_KSIZES
    for l in range(6):
        w = p[f"conv1d_{l + 1}/kernel"].float()
        fr, sw = fused.pack_conv_fragments_x3(w)
        nb = fr.numel() * 2
        assert torch.equal(blob[lay["woff"][l]: lay["woff"][l] + nb].view(torch.float16).reshape(fr.shape), fr)
        assert fused.pow2_exponent(float(w.abs().max() * 2.0 ** sw)) == 0  # max |W| 2^sw in [2^13, 2^14)
        back = fused.unpack_conv_fragments_x3(fr, sw, ks[l], ch[l], ch[l + 1])
        assert (back - w).abs().max() <= 2.0 ** -21 * w.abs().max()
        epi = blob[lay["eoff"][l]: lay["eoff"][l] + 4 * 8 * ch[l + 1]].view(torch.float32).reshape(8, ch[l + 1])
        scale, _ = fused.bn_affine(pooled, p, l + 1)
        torch.testing.assert_close(epi[0], scale * 2.0 ** -sw, rtol=0, atol=0)
