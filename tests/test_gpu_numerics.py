"""GPU: bit-exact scalar numerics of the tree kernels and the decode / gather kernels.

- glibc expf port (lzm_numerics.h) vs host libm expf on EVERY float in [-103.97, 0]
  (the domain of logit - max in CNode::expand, ctree_muzero/lib/cnode.cpp:129);
- glibc rand() jump-matrix generator vs the restatement pinned by libc vectors;
- Philox4x32-10 vs Random123 known answers;
- InverseScalarTransform kernel vs a torch fp32 restatement of scaling_transform.py:118-128
  (tolerance: rtol 1e-5, atol 1e-5 * support_scale — the fp32 summation-order bound);
- leaf gather vs torch advanced indexing (exact).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from lightzero_amd import _lib  # noqa: E402
from lightzero_amd._lib import call, ptr, stream_ptr  # noqa: E402
from oracle.oracle import glibc_rand_stream, lib as olib  # noqa: E402

DEV = torch.device("cuda", 0)


def dev_expf(bits_lo, n):
    b = torch.arange(bits_lo, bits_lo + n, dtype=torch.int64, device=DEV).to(torch.int32)
    x = b.view(torch.float32)
    out = torch.empty_like(x)
    call("lzm_debug_expf", ptr(x), ptr(out), n, stream_ptr())
    return out


def test_expf_port_exhaustive_negative_range():
    lo, hi = 0x80000000, 0xC2CFF1B4  # -0.0 .. -103.97 (below: glibc returns 0)
    chunk = 1 << 26
    threads = min(16, os.cpu_count() or 1)
    bad = 0
    for start in range(lo, hi + 1, chunk):
        n = min(chunk, hi + 1 - start)
        got = dev_expf(start - (1 << 32), n).cpu().numpy()
        bad += olib().lzo_expf_mismatches(start, n, got.ctypes.data, threads)
    assert bad == 0


def test_expf_port_special_values():
    xs = np.array([0.0, -0.0, 1.0, 10.0, 88.0, 88.72, 89.0, -88.0, -103.0, -104.0, -150.0, -np.inf, np.inf,
                   np.nan, 1e-30, -1e-30, 0.5, -0.5, 3.4e38, -3.4e38], np.float32)
    x = torch.from_numpy(xs).to(DEV)
    out = torch.empty_like(x)
    call("lzm_debug_expf", ptr(x), ptr(out), len(xs), stream_ptr())
    got = out.cpu().numpy()
    libm = ctypes.CDLL("libm.so.6")
    libm.expf.restype = ctypes.c_float
    libm.expf.argtypes = [ctypes.c_float]
    ref = np.array([libm.expf(float(v)) for v in xs], np.float32)
    assert np.array_equal(got.view(np.uint32)[~np.isnan(ref)], ref.view(np.uint32)[~np.isnan(ref)])
    assert np.isnan(got[np.isnan(ref)]).all()


@pytest.mark.parametrize("seed", [0, 1, 12345, 999999, 2147483646])
def test_device_glibc_stream(seed):
    n = 3000
    out = torch.empty(n, dtype=torch.int32, device=DEV)
    call("lzm_debug_glibc_rand", seed, n, ptr(out), stream_ptr())
    assert np.array_equal(out.cpu().numpy().astype(np.int64), glibc_rand_stream(seed, n))


def test_device_philox_known_answers():
    ck = np.array([[0, 0, 0, 0, 0, 0], [0xffffffff] * 6,
                   [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0]], np.uint32)
    d = torch.from_numpy(ck.view(np.int32)).to(DEV)
    out = torch.empty((3, 4), dtype=torch.int32, device=DEV)
    call("lzm_debug_philox", ptr(d), ptr(out), 3, stream_ptr())
    got = out.cpu().numpy().view(np.uint32)
    assert got.tolist() == [[0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8],
                            [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd],
                            [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]]


def test_dpp_butterflies_equal_shfl_xor():
    """lzm_tree.h's DPP / permlane xor_partner<D> picks lane ^ D for all 64 lanes and every D, and
    xor_sum / xor_max give the same bits as the __shfl_xor (ds_bpermute) butterflies they replaced"""
    rng = np.random.default_rng(7)
    for case in range(4):
        v = rng.normal(size=64).astype(np.float32) * np.float32(10.0 ** (case - 1))
        if case == 3:
            v[::3] = np.float32(-0.0)
        x = torch.from_numpy(v).to(DEV)
        out = torch.empty((16, 64), dtype=torch.float32, device=DEV)
        call("lzm_debug_xor", ptr(x), ptr(out), stream_ptr())
        o = out.cpu().numpy()
        lanes = np.arange(64)
        for k in range(6):
            want = v[lanes ^ (1 << k)]
            assert np.array_equal(o[k].view(np.uint32), want.view(np.uint32)), f"xor_partner<{1 << k}>"
            assert np.array_equal(o[6 + k].view(np.uint32), want.view(np.uint32)), f"__shfl_xor {1 << k}"
        assert np.array_equal(o[12].view(np.uint32), o[13].view(np.uint32)), "xor_sum"
        assert np.array_equal(o[14].view(np.uint32), o[15].view(np.uint32)), "xor_max"
        assert (o[14] == v.max()).all()


def torch_inverse_scalar_transform(logits, support_size, eps=0.001):
    """fp32 restatement of InverseScalarTransform.__call__ (scaling_transform.py:118-128)."""
    s = logits.sum(dim=1, keepdim=True)
    if torch.allclose(s, torch.ones_like(s), atol=1e-5):
        p = logits
    else:
        p = torch.softmax(logits, dim=1)
    support = torch.arange(-support_size, support_size + 1, dtype=torch.float64, device=logits.device)
    v = p.mul(support.unsqueeze(0)).sum(1, keepdim=True).float()
    tmp = ((torch.sqrt(1 + 4 * eps * (torch.abs(v) + 1 + eps)) - 1) / (2 * eps))
    return torch.sign(v) * (tmp * tmp - 1)


@pytest.mark.parametrize("rows,scale", [(256, 300), (64, 50), (7, 300)])
def test_inverse_scalar_transform_vs_torch(rows, scale):
    from lightzero_amd.scaling_transform import InverseScalarTransform
    g = torch.Generator(device="cpu").manual_seed(rows)
    logits = (torch.randn((rows, 2 * scale + 1), generator=g) * 3).to(DEV)
    logits[0, :] = -50.0
    logits[0, 2 * scale] = 50.0  # mass at +support
    got = InverseScalarTransform(scale, DEV)(logits)
    ref = torch_inverse_scalar_transform(logits, scale)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5 * scale)


def test_inverse_scalar_transform_skips_softmax_on_normalised_batch():
    from lightzero_amd.scaling_transform import InverseScalarTransform
    p = torch.softmax(torch.randn(32, 101), dim=1).to(DEV)
    got = InverseScalarTransform(50, DEV)(p)
    ref = torch_inverse_scalar_transform(p, 50)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5 * 50)


def test_inverse_scalar_transform_scalar_head():
    from lightzero_amd.scaling_transform import InverseScalarTransform
    v = (torch.randn(100, 1) * 20).to(DEV)
    got = InverseScalarTransform(300, DEV, categorical_distribution=False)(v)
    eps = 0.001
    tmp = ((torch.sqrt(1 + 4 * eps * (torch.abs(v) + 1 + eps)) - 1) / (2 * eps))
    torch.testing.assert_close(got, torch.sign(v) * (tmp * tmp - 1), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("row", [128, 1024, 7])
def test_gather_latent_exact(row):
    from lightzero_amd.tree import DeviceTree
    B, S = 96, 10
    t = DeviceTree(B, 2, S)
    pool = torch.randn((S + 1, B, row), device=DEV)
    x = torch.randint(0, S + 1, (B,), dtype=torch.int32, device=DEV)
    t.x.copy_(x)
    out = torch.empty((B, row), device=DEV)
    t.gather(pool, row, out)
    ref = pool[x.long(), torch.arange(B, device=DEV)]
    assert torch.equal(out, ref)
