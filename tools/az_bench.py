"""AlphaZero batched search throughput: 512 TicTacToe boards x 100 simulations,
the restated AlphaZeroModel (1 residual block, 16 channels; random-init heads). Prints one JSON line:
`value` = the fused search (one launch per search, network inside the kernel; HIP-event time too),
`generic_graph` = per-simulation tree kernel + torch network captured as one HIP graph, and two
reference-side rates timed on a bounded sample:
  - "reference_cpu": the reference's own compiled ctree (oracle/_ref/mcts_alphazero, built from the
    reference sources in the build container) driving the same network on the host CPU, one leaf
    per callback, like policy/alphazero.py:371-380 with a CPU device;
  - "reference_gpu": the same, with the network on this GPU (batch 1 per callback).

    python tools/az_bench.py [--boards 512] [--sims 100] [--searches 10] [--sample-boards 8]
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from lightzero_amd.alphazero import AlphaZeroMCTS, FusedAZNet  # noqa: E402
from lightzero_amd.model_az import tictactoe_alphazero_model  # noqa: E402
from oracle.tictactoe import SimTicTacToe, random_boards  # noqa: E402  (baseline leg only)


def device_rate(net, boards, starts, sims, searches, warmup):
    m = AlphaZeroMCTS(9, sims, 19652, 1.25, 0.3, 0.25, device="cuda", graph=True)
    with torch.no_grad():
        for _ in range(warmup):
            m.get_next_actions(boards, starts, net.compute_policy_value, 1.0, True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(searches):
            m.get_next_actions(boards, starts, net.compute_policy_value, 1.0, True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    return len(boards) * sims * searches / dt, dt / searches * 1e3


def fused_rate(net, boards, starts, sims, searches, warmup):
    """one launch per search (lzm_az_search_fused); timed with HIP events on the launch stream"""
    m = AlphaZeroMCTS(9, sims, 19652, 1.25, 0.3, 0.25, device="cuda")
    fnet = FusedAZNet(net)
    with torch.no_grad():
        for _ in range(warmup):
            m.search_fused(boards, starts, fnet, 1.0, True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(searches):
            m.search_fused(boards, starts, fnet, 1.0, True)
        e1.record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    return len(boards) * sims * searches / dt, dt / searches * 1e3, e0.elapsed_time(e1) / searches


def reference_rate(net, boards, starts, sims, device):
    """the reference ctree (compiled from /root/reference by oracle/build_ref.sh) with a per-leaf
    policy-value callback, as policy/alphazero.py:371-380 does it"""
    so = glob.glob(os.path.join(REPO, "oracle", "_ref", "mcts_alphazero*.so"))
    if not so:
        return None
    sys.path.insert(0, os.path.join(REPO, "oracle", "_ref"))
    import mcts_alphazero  # noqa: E402
    env = SimTicTacToe(scale=True)
    mcts = mcts_alphazero.MCTS(9, sims, 19652, 1.25, 0.3, 0.25, env)
    netd = net.to(device)

    def pv(e):
        legal = e.legal_actions
        _, scaled = e.current_state()
        x = torch.from_numpy(scaled).to(device=device, dtype=torch.float).unsqueeze(0)
        with torch.no_grad():
            probs, value = netd.compute_policy_value(x)
        return dict(zip(legal, probs.squeeze(0)[legal].detach().cpu().numpy())), value.item()

    t0 = time.perf_counter()
    for b, s in zip(boards, starts):
        cfg = dict(start_player_index=int(s), init_state=b.reshape(3, 3).astype(np.int32), katago_policy_init=False,
                   katago_game_state=None)
        mcts.get_next_action(cfg, pv, 1.0, True)
    dt = time.perf_counter() - t0
    return len(boards) * sims / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=512)
    ap.add_argument("--sims", type=int, default=100)
    ap.add_argument("--searches", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sample-boards", type=int, default=8)
    ap.add_argument("--no-reference", action="store_true")
    a = ap.parse_args()
    torch.manual_seed(0)
    net = tictactoe_alphazero_model().cuda()
    boards, starts = random_boards(a.boards, 0)
    frate, fms, fev = fused_rate(net, boards, starts, a.sims, max(a.searches, 20), a.warmup)
    rate, ms = device_rate(net, boards, starts, a.sims, a.searches, a.warmup)
    out = {"metric": "AlphaZero MCTS simulations/sec (TicTacToe, batched)", "value": frate, "unit": "sims/s",
           "ms_per_search": fms, "kernel_ms_per_search": fev,
           "generic_graph": {"value": rate, "ms_per_search": ms,
                             "what": "per-simulation tree kernel + torch network, one HIP graph per search"},
           "config": {"workload": "C4 tictactoe alphazero", "boards": a.boards, "num_simulations": a.sims,
                      "net": "AlphaZeroModel 1 resblock x 16 ch (random init, BN folded in the fused kernel)"}}
    if not a.no_reference:
        n = a.sample_boards
        torch.set_num_threads(1)
        cpu_net = tictactoe_alphazero_model()
        cpu_net.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
        r_cpu = reference_rate(cpu_net, boards[:n], starts[:n], a.sims, "cpu")
        r_gpu = reference_rate(net, boards[:n], starts[:n], a.sims, "cuda")
        out["reference_cpu"] = {"value": r_cpu, "cores": 1, "sample": f"{n} boards x {a.sims} sims"}
        out["reference_gpu"] = {"value": r_gpu, "sample": f"{n} boards x {a.sims} sims, batch-1 network on GPU"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
