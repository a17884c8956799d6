"""Diagnostic: per-phase shader-clock cycles of the fused AlphaZero search (config 4: 512 TicTacToe boards x
100 simulations), from the stamped instantiation that lzm_debug_az_stamps selects.

    python tools/az_phase_timing.py [--boards 512] [--sims 100] [--searches 5]

Prints cycles per workgroup per simulation for each phase (thread 0's view: a phase includes the barrier
waits that close it) and the event time of the stamped and the production launches.
LZM_AZ_BOARDS_PER_WG picks the boards per workgroup as in production.
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lightzero_amd import _lib  # noqa: E402
from lightzero_amd.alphazero import AlphaZeroMCTS, FusedAZNet  # noqa: E402
from lightzero_amd.model_az import tictactoe_alphazero_model  # noqa: E402
from oracle.tictactoe import random_boards  # noqa: E402  (input boards only)

NAMES = ["descend", "convolutions", "1x1 heads", "(unused)", "FC1/LayerNorm/FC2/softmax", "expand+backup"]


def timed(m, boards, starts, fnet, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        m.search_fused(boards, starts, fnet, 1.0, True)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=512)
    ap.add_argument("--sims", type=int, default=100)
    ap.add_argument("--searches", type=int, default=5)
    a = ap.parse_args()
    torch.manual_seed(0)
    net = tictactoe_alphazero_model().cuda().eval()
    boards, starts = random_boards(a.boards, 0)  # the bench's boards (tools/az_bench.py, bench.py config4)
    m = AlphaZeroMCTS(9, a.sims, 19652, 1.25, 0.3, 0.25, device="cuda")
    fnet = FusedAZNet(net)
    lib = _lib.load()
    with torch.no_grad():
        m.search_fused(boards, starts, fnet, 1.0, True)
        prod_ms = timed(m, boards, starts, fnet, 10)
        buf = torch.zeros(8, dtype=torch.int64, device="cuda")
        lib.lzm_debug_az_stamps(ctypes.c_void_p(buf.data_ptr()))
        m.search_fused(boards, starts, fnet, 1.0, True)
        torch.cuda.synchronize()
        buf.zero_()
        st_ms = timed(m, boards, starts, fnet, a.searches)
        lib.lzm_debug_az_stamps(None)
    v = buf.cpu().tolist()
    wgs_sims = v[7]  # sum over workgroups and searches of S
    wgs = wgs_sims / a.sims
    print(f"fused AlphaZero search, B={a.boards} S={a.sims}, workgroups x searches = {wgs:.0f}; "
          f"production {prod_ms * 1e3:.1f} us, stamped {st_ms * 1e3:.1f} us per search")
    print("cycles per workgroup per simulation (thread 0):")
    tot = 0.0
    for i, n in enumerate(NAMES):
        c = v[i] / wgs_sims
        tot += c
        print(f"  {n:24s} {c:9.0f}")
    print(f"  {'sum of phases':24s} {tot:9.0f}")
    kc = v[6] / wgs
    print(f"  kernel total per workgroup {kc:.0f} cycles = {kc / a.sims:.0f} per simulation; "
          f"implied clock {kc / (st_ms * 1e-3) / 1e9:.2f} GHz")


if __name__ == "__main__":
    main()
