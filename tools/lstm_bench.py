"""Microbenchmark: the EZ reward-LSTM step at Pong's shape (B = 256, K = 1536, H = 512):
lzm_ez_lstm_step (split-bf16 gate GEMM + cell, one launch) vs torch.addmm (rocBLAS f32) + lzm_ez_lstm_cell.

    python tools/lstm_bench.py [--envs 256] [--iters 200]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lightzero_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--K", type=int, default=1536)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--splitk", type=int, default=1, help="0: one workgroup per tile (no workspace)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, K, H = a.envs, a.K, a.H
    g = torch.Generator(device=dev).manual_seed(0)
    W = torch.randn(4 * H, K, generator=g, device=dev) * 0.03
    bias = torch.randn(4 * H, generator=g, device=dev) * 0.1
    xin = torch.randn(B, K, generator=g, device=dev)
    cpool = torch.randn(3, B, H, generator=g, device=dev)
    x = torch.randint(0, 3, (B,), generator=g, device=dev).to(torch.int32)
    slen = torch.randint(1, 9, (B,), generator=g, device=dev).to(torch.int32)
    L = _lib.load()
    frag = np.zeros(L.lzm_ez_lstm_frag_floats(K, H), np.float32)
    w = np.ascontiguousarray(W.cpu().numpy())
    _lib.check(L.lzm_ez_lstm_prepare(K, H, w.ctypes.data, frag.ctypes.data), "prepare")
    frag = torch.from_numpy(frag).to(dev)
    P = _lib.ptr
    outs = [torch.empty(B, H, device=dev) for _ in range(4)]
    ws = torch.zeros((L.lzm_ez_lstm_workspace_bytes(B, H) + 15) // 16 * 4, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)

    def fused():
        _lib.call("lzm_ez_lstm_step", B, K, H, P(xin), P(frag), P(bias), P(cpool), P(x), P(slen), 5, P(outs[0]),
                  P(outs[1]), P(outs[2]), P(outs[3]), P(ws) if a.splitk else None, P(err), _lib.stream_ptr())

    def blas():
        gates = torch.addmm(bias, xin, W.t())
        _lib.call("lzm_ez_lstm_cell", B, H, P(gates), P(cpool), P(x), P(slen), 5, P(outs[0]), P(outs[1]),
                  P(outs[2]), P(outs[3]), _lib.stream_ptr())

    res = {}
    for name, fn in (("fused", fused), ("rocblas+cell", blas)):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1e3 / a.iters
    # the two paths agree (f32-level error)
    fused()
    ref = [o.clone() for o in outs]
    blas()
    for r, o in zip(ref, outs):
        torch.testing.assert_close(r, o, rtol=2e-5, atol=2e-6)
    assert int(err.item()) == 0
    flops = 2.0 * B * K * 4 * H
    for name, us in res.items():
        print(f"{name:14s} {us:8.2f} us per step  ({flops / us / 1e6:.1f} TFLOP/s of f32 GEMM work)")


if __name__ == "__main__":
    main()
