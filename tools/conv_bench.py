"""Search throughput at the convolutional Atari configs (BASELINE.json configs 3 and 5, per GPU):
256 envs x 50 simulations through the drop-in EfficientZeroMCTSCtree (Pong: restated
EfficientZeroModel, 6 actions, LSTM 512, support 101) or MuZeroMCTSCtree (Breakout: restated
MuZeroModel, 4 actions, support 601), random-init weights with non-zero heads, synthetic frames.

Times `searches` full searches (root preparation + search + visit counts, inputs resident in HBM)
and prints one JSON line with sims/s and the network's roofline:
  - FLOPs per simulation from torch FlopCounterMode over one recurrent_inference at batch B, with the
    EfficientZero reward LSTM (FlopCounterMode does not see inside nn.LSTM) counted by hand:
    2 x 4H x (K + H) per row for the gate GEMM (K = reward planes, H = 512);
  - the matrix work runs split-bf16 (three bf16 terms per f32 operand, SIX bf16 products per f32
    product) on the bf16 MFMA pipe, so the bound is the dense BF16 peak (2.5 PF)
    against 6 x the convolution (+ LSTM gate) FLOPs; the f32-equivalent rate is reported beside;
and, with --cpu-baseline-secs > 0, the CPU baseline of the config (bench.cpu_baseline_conv: the
reference search loop over the oracle's bit-exact ctree with the same network on torch-CPU over the
host share, and on this GPU with per-simulation copies; plus the tree alone).

    python tools/conv_bench.py --kind ez|mz [--envs 256] [--sims 50] [--searches 5] [--graph 1]
                               [--precision bf16x3|f32] [--cpu-baseline-secs 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree  # noqa: E402
from lightzero_amd.model_conv import atari_efficientzero_model, atari_muzero_model  # noqa: E402
from lightzero_amd.utils import EasyDict  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3
BF16_PEAK_TFLOPS = 2500.0  # dense (MI355X_MICROARCH.md), not the 2:1-sparse figure


def recurrent_flops(model, kind, B, dev):
    """(all FLOPs, matrix-pipe FLOPs) per simulation row (bench.conv_flops_per_sim: FlopCounterMode over
    recurrent_inference plus, for EfficientZero, the reward LSTM's gate GEMM counted by hand)"""
    import bench
    return bench.conv_flops_per_sim(model, B, dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", choices=["ez", "mz"], default="ez")
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--searches", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--precision", choices=["split", "f32"], default=None,
                    help="native conv trunk precision (default: LZM_CONV_PRECISION or split)")
    ap.add_argument("--fused", type=int, default=1,
                    help="the one-launch search (lzm_search_conv / lzm_search_conv_ez) when it applies; 0: the generic path")
    ap.add_argument("--rng", choices=["glibc", "philox"], default="glibc",
                    help="tie-break stream: the reference's glibc rand() (parity) or per-root Philox")
    ap.add_argument("--cpu-baseline-secs", type=float, default=0.0,
                    help="> 0: also time the config's CPU baseline (bench.cpu_baseline_conv) for about this long")
    a = ap.parse_args()
    if a.precision:
        os.environ["LZM_CONV_PRECISION"] = a.precision
    precision = os.environ.get("LZM_CONV_PRECISION", "split")
    precision = "split" if precision == "bf16x3" else precision
    dev = torch.device("cuda", 0)
    B, S = a.envs, a.sims
    torch.manual_seed(0)
    model = (atari_efficientzero_model if a.kind == "ez" else atari_muzero_model)(last_linear_layer_init_zero=False)
    model = model.to(dev).eval()
    A = model.action_space_size
    scale = 50 if a.kind == "ez" else 300
    cls = EfficientZeroMCTSCtree if a.kind == "ez" else MuZeroMCTSCtree
    cls.rng_mode = a.rng
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=dev, lstm_horizon_len=5,
                        use_hip_graph=bool(a.graph), fused_search=bool(a.fused),
                        model=dict(support_scale=scale, categorical_distribution=True)))
    mcts = cls(cfg)
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.integers(0, 256, size=(B, 4, 64, 64)).astype(np.float32) / 255.0).to(dev)
    noises = torch.from_numpy(rng.dirichlet([0.3] * A, size=B).astype(np.float32)).to(dev)
    legal = [list(range(A))] * B
    to_play = torch.full((B,), -1, dtype=torch.int32, device=dev)
    rewards = torch.zeros(B, dtype=torch.float32, device=dev)
    seeds = torch.arange(S, dtype=torch.int32, device=dev)
    with torch.no_grad():
        out = model.initial_inference(obs)
    roots = cls.roots(B, legal)

    def one():
        roots.prepare_device(0.25, noises, rewards, out.policy_logits.float(), to_play)
        if a.kind == "ez":
            mcts.search(roots, model, out.latent_state, out.reward_hidden_state, to_play, seeds=seeds)
        else:
            mcts.search(roots, model, out.latent_state, to_play, seeds=seeds)
        return roots.tree.distributions()

    for _ in range(a.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.searches):
        d = one()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.searches
    assert int(d.sum()) == B * S
    roots.tree.check_errors()
    fused = (mcts._fused_conv(model, roots.tree, (64, 8, 8)) if a.kind == "mz" else
             mcts._fused_conv(model, roots.tree, (64, 8, 8), model.lstm_hidden_size)) is not None
    flops, matrix = recurrent_flops(model, a.kind, B, dev)
    net_tflops = flops * B * S / dt / 1e12
    split = precision == "split"
    # split: the trunk's convolutions and EZ's LSTM gate GEMM at 3 fp16 products per f32 product
    mfma = (3.0 if split else 1.0) * matrix * B * S / dt / 1e12
    peak = BF16_PEAK_TFLOPS if split else FP32_MFMA_PEAK_TFLOPS
    cpu = None
    if a.cpu_baseline_secs > 0:
        import bench
        cpu = bench.cpu_baseline_conv(a.kind, B, S, model, a.cpu_baseline_secs, dev)
    print(json.dumps({
        "metric": "MCTS simulations/sec", "value": B * S / dt, "unit": "sims/s", "ms_per_search": dt * 1e3,
        "config": {"workload": "C3 Pong EfficientZero" if a.kind == "ez" else "C5 Breakout MuZero (per GPU)",
                   "envs": B, "num_simulations": S, "actions": A, "support": 2 * scale + 1, "latent": [64, 8, 8],
                   "path": ("one-launch search (lzm_search_conv%s)" % ("_ez" if a.kind == "ez" else "")) if fused else
                   "generic (HIP tree kernels + PyTorch-ROCm network)", "hip_graph": bool(a.graph) and not fused,
                   "conv_precision": precision, "rng": a.rng},
        "net_flops_per_sim": flops, "matrix_flops_per_sim": matrix, "net_tflops_whole_search": net_tflops,
        "roofline": {"bound": "mfma", "pipe": "bf16 MFMA, 6 products per f32 product (split-bf16)" if split else
                     "f32 MFMA (exact f32)", "achieved": round(mfma, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(mfma / peak, 4), "f32_equivalent_tflops": round(net_tflops, 2),
                     "f32_equivalent_frac_of_fp32_peak": round(net_tflops / FP32_MFMA_PEAK_TFLOPS, 4)},
        "cpu_baseline": cpu, "vs_cpu_baseline": (B * S / dt) / cpu["value"] if cpu else None}))


if __name__ == "__main__":
    main()
