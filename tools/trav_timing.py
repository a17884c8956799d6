"""Phase timing of the generic path's look-back traverse (LZM_PHASE_TIMING=1 selects the stamped
instantiation, one root per workgroup): shader cycles per root per launch in the setup, the draw-free
walk, the look-back + draws, and the outputs, at a conv config (Breakout MZ / Pong EZ, 256 x 50).

    LZM_PHASE_TIMING=1 python tools/trav_timing.py --kind mz
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from lightzero_amd import _lib  # noqa: E402
from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree  # noqa: E402
from lightzero_amd.model_conv import atari_efficientzero_model, atari_muzero_model  # noqa: E402
from lightzero_amd.utils import EasyDict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", choices=["ez", "mz"], default="mz")
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--sims", type=int, default=50)
    a = ap.parse_args()
    assert os.environ.get("LZM_PHASE_TIMING") == "1", "set LZM_PHASE_TIMING=1"
    dev = torch.device("cuda", 0)
    B, S = a.envs, a.sims
    torch.manual_seed(0)
    model = (atari_efficientzero_model if a.kind == "ez" else atari_muzero_model)(last_linear_layer_init_zero=False)
    model = model.to(dev).eval()
    A = model.action_space_size
    scale = 50 if a.kind == "ez" else 300
    cls = EfficientZeroMCTSCtree if a.kind == "ez" else MuZeroMCTSCtree
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=dev, lstm_horizon_len=5,
                        use_hip_graph=False, model=dict(support_scale=scale, categorical_distribution=True)))
    mcts = cls(cfg)
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.integers(0, 256, size=(B, 4, 64, 64)).astype(np.float32) / 255.0).to(dev)
    noises = torch.from_numpy(rng.dirichlet([0.3] * A, size=B).astype(np.float32)).to(dev)
    to_play = torch.full((B,), -1, dtype=torch.int32, device=dev)
    rewards = torch.zeros(B, dtype=torch.float32, device=dev)
    seeds = torch.arange(S, dtype=torch.int32, device=dev)
    with torch.no_grad():
        out = model.initial_inference(obs)
    roots = cls.roots(B, [list(range(A))] * B)

    def one():
        roots.prepare_device(0.25, noises, rewards, out.policy_logits.float(), to_play)
        if a.kind == "ez":
            mcts.search(roots, model, out.latent_state, out.reward_hidden_state, to_play, seeds=seeds)
        else:
            mcts.search(roots, model, out.latent_state, to_play, seeds=seeds)

    one()
    torch.cuda.synchronize()
    L = _lib.load()
    buf = (ctypes.c_uint64 * 64)()
    L.lzm_debug_phase_cycles(roots.tree.h, buf, 1)
    n = 3
    for _ in range(n):
        one()
    torch.cuda.synchronize()
    L.lzm_debug_phase_cycles(roots.tree.h, buf, 0)
    v = np.array(buf[32:39], dtype=np.float64)
    roots_n = max(v[4], 1)
    names = ["setup", "draw-free walk", "look-back + draws", "outputs"]
    print(f"look-back traverse, {a.kind}, B={B}, S={S}: cycles per root per launch")
    for k, name in enumerate(names):
        print(f"  {name:20s} {v[k] / roots_n:10.0f}")
    print(f"  roots needing a draw: {v[5] / roots_n * 100:.1f}%   max start->done: {v[6]:.0f} cycles")


if __name__ == "__main__":
    main()
