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
    ap.add_argument("--no-check", action="store_true", help="diagnostic builds (results invalid)")
    ap.add_argument("--stamps", action="store_true", help="print per-phase shader clocks of one launch")
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
    # the rows' split scales (lzm_conv.h ls_row_exp of each row's max)
    xscale = torch.tensor([14 - int(np.floor(np.log2(max(float(v), 1.0)))) for v in xin.abs().amax(dim=1).cpu()],
                          dtype=torch.int32, device=dev)

    def fused():
        _lib.call("lzm_ez_lstm_step", B, K, H, P(xin), P(xscale), P(frag), P(bias), P(cpool), P(x), P(slen), 5,
                  P(outs[0]), P(outs[1]), P(outs[2]), P(outs[3]), P(ws) if a.splitk else None, P(err), None,
                  _lib.stream_ptr())

    def blas():
        gates = torch.addmm(bias, xin, W.t())
        _lib.call("lzm_ez_lstm_cell", B, H, P(gates), P(cpool), P(x), P(slen), 5, P(outs[0]), P(outs[1]),
                  P(outs[2]), P(outs[3]), _lib.stream_ptr())

    res = {}
    for name, fn in (("fused", fused), ("rocblas+cell", blas)):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        # 20 steps captured in one HIP graph (no host launch cost in the timing)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(20):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = max(1, a.iters // 20)
        e0.record()
        for _ in range(n):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1e3 / (20 * n)
    # the two paths agree (f32-level error)
    fused()
    ref = [o.clone() for o in outs]
    blas()
    if not a.no_check:
        for r, o in zip(ref, outs):
            torch.testing.assert_close(r, o, rtol=1e-4, atol=1e-5)
        assert int(err.item()) == 0
    if a.stamps:
        # per-block real-time stamps (100 MHz) of one launch: prologue, stage loop, hand-off, epilogue
        st = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
        L.lzm_debug_lstm_stamps(P(st))
        torch.cuda.synchronize()
        for _ in range(50):  # back to back (a launch after an idle GPU runs at low clocks); the last one wins
            fused()
        torch.cuda.synchronize()
        L.lzm_debug_lstm_stamps(None)
        v = st.view(-1, 8).cpu().numpy().astype(np.float64)
        v = v[v[:, 0] > 0]
        t0 = v[:, 0].min()
        nblk = len(v)
        up = v[: nblk // 2] if a.splitk else v[:0]
        lo = v[nblk // 2:] if a.splitk else v
        for name, w in (("upper K half", up), ("lower K half", lo)):
            if len(w) == 0:
                continue
            us = lambda x: f"{np.mean(x) * 0.01:.2f}"  # 100 MHz ticks -> us
            end = np.max(w[:, 3:5], axis=1)
            print(f"{name} (us, mean over blocks): start {us(w[:, 0] - t0)}  prologue {us(w[:, 1] - w[:, 0])}  "
                  f"stages {us(w[:, 2] - w[:, 1])}  hand-off {us(w[:, 3] - w[:, 2])}  end {us(end - t0)}  "
                  f"last end {np.max(end - t0) * 0.01:.2f}")
    flops = 2.0 * B * K * 4 * H
    for name, us in res.items():
        print(f"{name:14s} {us:8.2f} us per step  ({flops / us / 1e6:.1f} TFLOP/s of f32 GEMM work)")


if __name__ == "__main__":
    main()
