"""CPU: the C-ABI library loads and exports every entry point include/lzmcts.h declares; the
product path refuses to run without a GPU (no CPU fallback)."""
import os
import re

import pytest

from lightzero_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "lzmcts.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lzm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_core_entry_points():
    syms = declared_symbols()
    for s in ("lzm_create", "lzm_traverse", "lzm_backprop", "lzm_decode_backprop", "lzm_gather_latent",
              "lzm_roots_prepare", "lzm_get_distributions", "lzm_get_values", "lzm_get_trajectories"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_binding_table_matches_header():
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from lightzero_amd.tree import DeviceTree
    with pytest.raises(_lib.LzmError):
        DeviceTree(4, 2, 8)


def test_module_api_type_errors_match_cython():
    from lightzero_amd.ctree import mz_tree
    roots = mz_tree.Roots(2, [[0, 1], [0, 1]])
    with pytest.raises(TypeError):
        roots.prepare(0.25, ((0.5, 0.5), (0.5, 0.5)), [0.0, 0.0], [[0.0, 0.0], [0.0, 0.0]], [-1, -1])
    with pytest.raises(TypeError):
        roots.prepare_no_noise([0.0, 0.0], "not-a-list", [-1, -1])


def test_easydict_semantics():
    from lightzero_amd.utils import EasyDict
    d = EasyDict(dict(a=1, model=dict(support_scale=300)))
    assert d.model.support_scale == 300
    d.update(dict(b=2))
    assert d.b == 2


def _row_exp(W):
    """lzm_conv.h's weight-row exponent: 14 - floor(log2 max |row|), clamped to +-24 (0 for a zero row)"""
    import numpy as np
    m = np.abs(W).max(axis=1).astype(np.float32)
    e = 14 - (((m.view(np.uint32) >> 23) & 0xFF).astype(np.int64) - 127)
    return np.where(m > 0, np.clip(e, -24, 24), 0)


def test_split_trunk_packing_recovers_f32_weights():
    """lzm_conv_trunk_prepare_p(LZM_CONV_SPLIT) (host code, no GPU): every out channel's row is packed scaled by
    2^e_c (its largest |w| in [2^14, 2^15)), the packed two fp16 terms h + l give back W 2^e_c within 2^-22
    relative (2^-25 absolute below fp16's normal range, i.e. 2^-17 below the row's max), h is the
    round-to-nearest fp16, and the [wave][chunk][term][lane][8] fragment map puts W[out][in][tap] where the
    16x16x32 B operand expects it (out 16 wave + lane % 16, in 32 j + 8 (lane / 16) + e, chunk 2 tap + j). The
    layer's scales 2^-e_c and bounds {max row L1 norm, max |bias|} follow the fragments; weights spanning
    1e-4 .. 1e3 (the range the unscaled split lost) come back the same way."""
    import ctypes
    import numpy as np
    L = _lib.load()
    n_dres, n_pres, r_ch, h_ch = 1, 1, 16, 32
    W3 = 64 * 64 * 9
    nraw = W3 + n_dres * 2 * (W3 + 64) + r_ch * 64 + r_ch + n_pres * 2 * (W3 + 64) + h_ch * 64 + h_ch
    rng = np.random.default_rng(0)
    n = L.lzm_conv_trunk_floats_p(n_dres, n_pres, 1)
    assert n > 0 and L.lzm_conv_trunk_floats_p(n_dres, n_pres, 7) < 0
    n3 = 1 + 2 * (n_dres + n_pres)
    for spread in (False, True):
        raw = (rng.standard_normal(nraw) * 0.05).astype(np.float32)
        if spread:  # rows from 1e-4 to 1e3
            raw[:W3] *= np.repeat(np.logspace(-4, 3, 64), 64 * 9).astype(np.float32) / 0.05
        out = np.zeros(n, np.float32)
        assert L.lzm_conv_trunk_prepare_p(1, n_dres, n_pres, r_ch, h_ch, ctypes.c_void_p(raw.ctypes.data),
                                          ctypes.c_void_p(out.ctypes.data)) == 0
        u = out.view(np.uint16)[: 4 * 18 * 2 * 64 * 8].reshape(4, 18, 2, 64, 8)  # dynamics conv blob
        terms = u.view(np.float16).astype(np.float64)
        rec = terms.sum(axis=2)  # [w][s][lane][e]
        Wf = raw[:W3].reshape(64, 64 * 9)
        e = _row_exp(Wf)
        W = Wf.astype(np.float64).reshape(64, 64, 9) * np.exp2(e)[:, None, None]
        w_, s_, l_, e_ = np.meshgrid(np.arange(4), np.arange(18), np.arange(64), np.arange(8), indexing="ij")
        cout = 16 * w_ + (l_ & 15)
        cin = 32 * (s_ & 1) + 8 * (l_ >> 4) + e_
        want = W[cout, cin, s_ >> 1]
        assert np.abs(want).max() < 2.0 ** 15
        # two fp16 terms: 22 significand bits; below fp16's normal range an absolute 2^-25
        assert np.all(np.abs(rec - want) <= np.abs(want) * 2.0 ** -22 + 2.0 ** -25)
        hi = terms[:, :, 0]
        assert np.all(np.abs(hi - want) <= np.abs(want) * 2.0 ** -11 + 2.0 ** -25)
        sc = out[n - (n3 + 2) * 68: n - (n3 + 2) * 4].reshape(n3 + 2, 64)
        bd = out[n - (n3 + 2) * 4:].reshape(n3 + 2, 4)
        assert np.array_equal(sc[0], np.exp2(-e).astype(np.float32))
        assert bd[0, 0] >= np.abs(Wf.astype(np.float64)).sum(axis=1).max() and bd[0, 1] == 0
        # the first block's conv 1: bias bound max |b1|
        b1 = raw[W3 + W3: W3 + W3 + 64]
        assert bd[1, 1] >= np.abs(b1).max() and bd[1, 1] <= np.abs(b1).max() * (1 + 1e-5)
    assert L.lzm_conv_trunk_actmap_bound(n_dres, n_pres, 3.5, ctypes.c_void_p(out.ctypes.data)) == 0
    assert out[n - (n3 + 2) * 4 + 1] >= 3.5


def test_lstm_gate_fragments_recover_f32_weights():
    """lzm_ez_lstm_prepare (host code, no GPU): the [n-block][wave][chunk][term][lane][8] split-fp16
    fragments of the LSTM gate weights W [4H][K] give back W (h + l within 2^-22 relative, 2^-25 absolute
    below fp16's normal range) at the
    place the fused gate-GEMM + cell kernel reads it: lane l of wave w in n-block nb is column l % 16 =
    4 u + gate of unit 16 nb + 4 w + u (torch row gate * H + unit), k = 32 chunk + 8 (l / 16) + e"""
    import ctypes
    import numpy as np
    L = _lib.load()
    K, H = 128, 32
    assert L.lzm_ez_lstm_frag_floats(K, H) == K * 4 * H * 2 // 2 + 4 * H  # fragments, then the column scales
    assert L.lzm_ez_lstm_frag_floats(100, H) < 0 and L.lzm_ez_lstm_frag_floats(K, 24) < 0
    rng = np.random.default_rng(1)
    W = (rng.standard_normal((4 * H, K)) * np.logspace(-3, 2, 4 * H)[:, None]).astype(np.float32)
    out = np.zeros(L.lzm_ez_lstm_frag_floats(K, H), np.float32)
    assert L.lzm_ez_lstm_prepare(K, H, ctypes.c_void_p(W.ctypes.data), ctypes.c_void_p(out.ctypes.data)) == 0
    nb_n, nch = H // 16, K // 32
    e = _row_exp(W)
    assert np.array_equal(out[K * 4 * H:], np.exp2(-e).astype(np.float32))
    u = out[:K * 4 * H].view(np.uint16).reshape(nb_n, 4, nch, 2, 64, 8)
    rec = u.view(np.float16).astype(np.float64).sum(axis=3)  # [nb][w][j][lane][e]
    nb_, w_, j_, l_, e_ = np.meshgrid(np.arange(nb_n), np.arange(4), np.arange(nch), np.arange(64), np.arange(8),
                                      indexing="ij")
    n = l_ & 15
    unit = 16 * nb_ + 4 * w_ + (n >> 2)
    want = (W.astype(np.float64) * np.exp2(e)[:, None])[(n & 3) * H + unit, 32 * j_ + 8 * (l_ >> 4) + e_]
    assert np.all(np.abs(rec - want) <= np.abs(want) * 2.0 ** -22 + 2.0 ** -25)


def test_representation_entry_points_validate_arguments_on_the_host():
    """lzm_bias_add_relu / lzm_conv_resnet8_p (conv_infer.FoldedConvInitial's kernels) refuse bad
    shapes and alignments before any HIP call (status LZM_ERR_ARG, no launch, no GPU needed)"""
    import ctypes
    L = _lib.load()
    err = -1  # LZM_ERR_ARG
    buf = ctypes.create_string_buffer(64 + 16)
    base = ctypes.addressof(buf)
    p16 = ctypes.c_void_p((base + 15) & ~15)  # 16-B aligned
    p4 = ctypes.c_void_p(((base + 15) & ~15) + 4)  # misaligned
    assert L.lzm_bias_add_relu(None, p16, None, 1, 1, 4, 1, None) == err
    assert L.lzm_bias_add_relu(p16, p16, None, 1, 1, 6, 1, None) == err  # HW % 4
    assert L.lzm_bias_add_relu(p4, p16, None, 1, 1, 4, 1, None) == err  # alignment
    assert L.lzm_conv_resnet8_p(1, 0, 1, 16, p16, p16, p16, p16, None, None) == err  # no residual block
    assert L.lzm_conv_resnet8_p(1, 9, 1, 16, p16, p16, p16, p16, None, None) == err  # more than 8
    assert L.lzm_conv_resnet8_p(1, 2, 1, 33, p16, p16, p16, p16, None, None) == err  # head channels
    assert L.lzm_conv_resnet8_p(1, 2, 1, 16, p16, p4, p16, p16, None, None) == err  # input alignment
