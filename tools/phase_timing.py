"""Diagnostic: per-phase shader-clock cycles of the fused search kernel (LZM_PHASE_TIMING=1).

    LZM_PHASE_TIMING=1 python tools/phase_timing.py [--envs 256] [--sims 50] [--zero-heads] [--roots R]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LZM_PHASE_TIMING", "1")

import bench  # noqa: E402
from lightzero_amd import _lib  # noqa: E402

NAMES = ["select", "offsets+lookback", "gather", "dynamics", "reward head+decode", "pred trunk",
         "value head+decode", "policy head", "file latents", "expand+backup", "stage-in", "write-back",
         "select terms (res)", "walk (res, of select)", "expand (res, of e+b)", "support logits (res)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--rng", default="glibc")
    ap.add_argument("--zero-heads", action="store_true")
    ap.add_argument("--roots", type=int, default=0, help="roots per workgroup (0: library's choice)")
    a = ap.parse_args()
    if a.roots:
        os.environ["LZM_ROOTS_PER_WG"] = str(a.roots)
    R = a.roots or next(r for r in (1, 2, 4, 8) if -(-a.envs // r) <= 256 or r == 8)
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, a.zero_heads, 0)
    step = bench.GpuStep(a.envs, a.sims, model, dev, a.rng, 0, 1)
    step()
    torch.cuda.synchronize()
    from lightzero_amd.tree import POOL
    t = next(iter(POOL._free.values()))[0]
    buf = (ctypes.c_uint64 * 64)()
    _lib.load().lzm_debug_phase_cycles(t.h, buf, 1)
    _lib.load().lzm_debug_root_wait_cycles(t.h, buf, 0, 1)
    n = 3
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    _lib.load().lzm_debug_phase_cycles(t.h, buf, 0)
    G = -(-a.envs // R)
    per = np.array(buf[:16], dtype=np.float64) / (n * G)
    tot = per.sum()
    print(f"per workgroup per search (cycles), R={R}, G={G}, sims={a.sims}:")
    for name, c in zip(NAMES, per):
        print(f"  {name:20s} {c:12.0f}  per-sim {c / a.sims:9.0f}  {100 * c / tot:5.1f}%")
    print(f"  total {tot:.0f} cycles = {tot / 2.1e3:.0f} us at 2.1 GHz")
    sub = np.array(buf[16:64], dtype=np.float64) / (n * G * a.sims)
    print("sub-stamps per simulation (cycles; index = stamp id - 16, meaning per kernel):")
    print("  " + "  ".join(f"{q}:{c:.0f}" for q, c in enumerate(sub) if c > 0))
    # per-workgroup look-back wait (resident kernel, parity mode): by root range and by XCD (g % 8)
    wait = (ctypes.c_uint64 * 1024)()
    _lib.load().lzm_debug_root_wait_cycles(t.h, wait, 1024, 0)
    w = np.array(wait[:G], dtype=np.float64) / (n * a.sims)
    if w.sum() > 0:
        print("look-back wait per simulation (cycles), by root range:")
        for q in range(8):
            lo, hi = q * G // 8, (q + 1) * G // 8
            print(f"  roots {lo:4d}-{hi - 1:4d}: mean {w[lo:hi].mean():7.0f}  max {w[lo:hi].max():7.0f}")
        print("by XCD (g % 8): " + "  ".join(f"{x}:{w[x::8].mean():.0f}" for x in range(8)))
        print("roots 0-7: " + "  ".join(f"{x}:{w[x]:.0f}" for x in range(min(8, G))))


if __name__ == "__main__":
    main()
