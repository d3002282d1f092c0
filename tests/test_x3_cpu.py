"""CPU tier of the fp32-faithful engine (ops/x3.py): fragment packing and the fp16x3 split."""
import torch

from uncertaintyquantification_sleepapnea_1dcnn_amd.models import reference as R
from uncertaintyquantification_sleepapnea_1dcnn_amd.models.spec import DEFAULT_SPEC as SPEC
from uncertaintyquantification_sleepapnea_1dcnn_amd.ops import x3


def test_pack_roundtrip_is_fp32_faithful():
    p = R.synthetic_params(SPEC, 4)
    ch, ks = SPEC.channels(), [b.kernel_size for b in SPEC.blocks]
    for l in range(1, 6):
        w = p[f"conv1d_{l + 1}/kernel"]
        fr, sc = x3.pack_conv(w)
        assert fr.dtype == torch.float16 and fr.numel() == ks[l] * ch[l] * ch[l + 1] * 2
        back = x3.unpack_conv(fr, sc, ks[l], ch[l], ch[l + 1])
        # relative for every weight above 2^-8 of the largest (below, the lo half is subnormal: absolute error)
        floor = w.double().abs().max() * 2 ** -8
        rel = ((back.double() - w.double()).abs() / w.double().abs().clamp_min(floor)).max().item()
        assert rel < 2 ** -21, f"block {l + 1}: hi+lo relative error {rel:.2e}"
        # both halves in the fp16 normal range (no overflow, lo not flushed for the large weights)
        assert torch.isfinite(fr.float()).all()
        assert fr.float().abs().max().item() < 2 ** 14


def test_fragment_layout_matches_mfma_a_map():
    """lane l of fragment (chunk c, tap j, ct) holds W[j][32c + 8(l>>4) + e][16ct + (l&15)]."""
    k, cin, cout = 3, 64, 32
    w = torch.arange(k * cin * cout, dtype=torch.float32).reshape(k, cin, cout) / 4096.0
    fr, sc = x3.pack_conv(w)
    v = fr.reshape(cin // 32, k, cout // 16, 2, 64, 8)
    for (c, j, ct, l, e) in [(0, 0, 0, 0, 0), (1, 2, 1, 37, 5), (0, 1, 1, 63, 7), (1, 0, 0, 16, 3)]:
        want = w[j, 32 * c + 8 * (l >> 4) + e, 16 * ct + (l & 15)].item()
        got = (v[c, j, ct, 0, l, e].float() + v[c, j, ct, 1, l, e].float()).item() * sc
        assert abs(got - want) <= 1e-6 * max(1.0, abs(want))


def test_emulated_x3_conv_is_fp32_accurate():
    """The three-product split reproduces an fp64 convolution to ~fp32 precision (it is the arithmetic
    the layer kernel performs, up to fp32 accumulation order)."""
    g = torch.Generator().manual_seed(0)
    h = torch.randn(5, 60, 96, generator=g, dtype=torch.float64)
    p = R.synthetic_params(SPEC, 1)
    w = p["conv1d_5/kernel"]
    fr, sc = x3.pack_conv(w)
    y = x3.emulate_conv(h.float().double(), fr, sc, 9, 96, 256)
    ref = R.conv1d_same(h.float().double(), w.double(), torch.zeros(256, dtype=torch.float64))
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    assert err < 3e-7, err


def test_mask_side_selection(monkeypatch):
    """ops/x3.py: layer l draws block l+1's mask in its epilogue (sign_out) iff l is listed, and layer l+1
    then decodes it (sign_in); the pass-shared block-1 output (layer 1's input) is always hashed."""
    monkeypatch.setenv("APNEAUQ_X3_SIGN_MASK", "1, 3,4")
    sl = x3._sign_layers()
    assert sl == frozenset({1, 3, 4})
    assert [x3._sign(l, sl) for l in range(1, 6)] == [(False, True), (True, False), (False, True), (True, True),
                                                      (True, False)]
    monkeypatch.setenv("APNEAUQ_X3_SIGN_MASK", "")
    assert x3._sign_layers() == frozenset()
    monkeypatch.delenv("APNEAUQ_X3_SIGN_MASK")
    assert x3._sign_layers() == frozenset(int(t) for t in x3._SIGN_DEFAULT.split(","))
    # layer 5 (block 6) never stores its mask: it reduces its masked output in place
    assert x3._sign(5, frozenset({5}))[1] is False
