"""Diagnostic: per-phase shader-clock cycles of the one-launch conv searches (lzm_search_conv /
lzm_search_conv_ez, LZM_PHASE_TIMING=1 selects their stamped instantiations).

    python tools/conv_phase_timing.py [--kind mz|ez] [--envs 256] [--sims 50] [--rng glibc|philox]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LZM_PHASE_TIMING"] = "1"

from lightzero_amd import _lib  # noqa: E402
from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree  # noqa: E402
from lightzero_amd.model_conv import atari_efficientzero_model, atari_muzero_model  # noqa: E402
from lightzero_amd.utils import EasyDict  # noqa: E402

NAMES = ["selection (+look-back)", "trunk input", "trunk layers", "head hidden", "head outputs", "decode",
         "expand+backup"]
NAMES_EZ = ["selection (+look-back)", "trunk input", "trunk layers", "value/policy hidden",
            "value/policy out + decode", "LSTM tile (+waits)", "value-prefix head (+wait)", "expand+backup"]
WAITS_EZ = ["late look-back", "kernel total", "wait: tile rows (xin)", "wait: upper K half", "wait: row's tiles",
            "gate GEMM"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", choices=["mz", "ez"], default="mz")
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--rng", default="glibc")
    ap.add_argument("--searches", type=int, default=3)
    ap.add_argument("--no-check", action="store_true", help="skip the error words (diagnostic builds)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, S = a.envs, a.sims
    torch.manual_seed(0)
    ez = a.kind == "ez"
    model = (atari_efficientzero_model if ez else atari_muzero_model)(last_linear_layer_init_zero=False).to(dev).eval()
    A = model.action_space_size
    cls = EfficientZeroMCTSCtree if ez else MuZeroMCTSCtree
    cls.rng_mode = a.rng
    mcts = cls(EasyDict(dict(num_simulations=S, discount_factor=0.997, device=dev, lstm_horizon_len=5,
                             model=dict(support_scale=50 if ez else 300, categorical_distribution=True))))
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.integers(0, 256, size=(B, 4, 64, 64)).astype(np.float32) / 255.0).to(dev)
    noises = torch.from_numpy(rng.dirichlet([0.3] * A, size=B).astype(np.float32)).to(dev)
    to_play = torch.full((B,), -1, dtype=torch.int32, device=dev)
    rewards = torch.zeros(B, dtype=torch.float32, device=dev)
    seeds = torch.arange(S, dtype=torch.int32, device=dev)
    with torch.no_grad():
        out = model.initial_inference(obs)
    roots = cls.roots(B, [list(range(A))] * B)
    buf = (ctypes.c_uint64 * 64)()

    def one():
        roots.prepare_device(0.25, noises, rewards, out.policy_logits.float(), to_play)
        if ez:
            mcts.search(roots, model, out.latent_state, out.reward_hidden_state, to_play, seeds=seeds)
        else:
            mcts.search(roots, model, out.latent_state, to_play, seeds=seeds)

    one()
    torch.cuda.synchronize()
    fz = mcts._fused_conv(model, roots.tree, (64, 8, 8), *((model.lstm_hidden_size,) if ez else ()))
    assert fz is not None, "not the one-launch search"
    _lib.load().lzm_debug_phase_cycles(roots.tree.h, buf, 1)
    for _ in range(a.searches):
        one()
    torch.cuda.synchronize()
    _lib.load().lzm_debug_phase_cycles(roots.tree.h, buf, 0)
    if not a.no_check:
        roots.tree.check_errors()
    if ez:
        per = np.array(buf[40:54], dtype=np.float64) / (a.searches * B)
        print(f"one-launch EZ search, per workgroup (root) per simulation, cycles (B={B}, S={S}, rng={a.rng}):")
        tot = per[:8].sum()
        for name, c in zip(NAMES_EZ, per[:8]):
            print(f"  {name:28s} {c / S:9.0f}  {100 * c / tot:5.1f}%")
        for name, c in zip(WAITS_EZ, per[8:14]):
            print(f"  {name:28s} {c / S:9.0f}")
        return
    per = np.array(buf[40:53], dtype=np.float64) / (a.searches * B)
    print(f"one-launch conv search, per workgroup (root) per simulation, cycles (B={B}, S={S}, rng={a.rng}):")
    tot = per[:7].sum()
    for name, c in zip(NAMES, per[:7]):
        print(f"  {name:24s} {c / S:9.0f}  {100 * c / tot:5.1f}%")
    print(f"  sum of phases per sim {tot / S:.0f}; kernel total per root {per[7]:.0f} cycles "
          f"(per sim {per[7] / S:.0f}); late-draw look-back per sim {per[8] / S:.0f}; classification walk per "
          f"sim {per[10] / S:.0f} (of selection), levels per sim {per[11] / S:.2f}, late-draw ties per sim "
          f"{per[12] / S:.2f}")


if __name__ == "__main__":
    main()
