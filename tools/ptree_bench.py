"""BASELINE.json config 1: CartPole MuZero with the pure-Python tree (ptree), 8 envs x 25 sims, MLP on CPU.

The reference times `MuZeroMCTSPtree.search` (lzero/mcts/tree_search/mcts_ptree.py:92-194) over
lzero/mcts/ptree/ptree_mz.py. On the GPU box the reference does not exist, so this times the
restatement oracle/ptree_port.py — checked transcript-exact against the reference's own ptree
(tests/test_ptree_port.py) — with the same MuZeroModelMLP on torch-CPU and InverseScalarTransform:
per search, initial_inference, Roots.prepare with Dirichlet noise, and S simulations of
batch_traverse -> host gather of latent[x][y] -> recurrent_inference -> inverse transform ->
batch_backpropagate. `--reference` (build container only) runs the same loop over the reference's
ptree_mz.py itself (loaded by file path) for the reference / port calibration.

    python tools/ptree_bench.py [--envs 8] [--sims 25] [--secs 10] [--threads 1] [--reference]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from oracle import ptree_port as pp  # noqa: E402


def inverse(logits, support):
    p = torch.softmax(logits, dim=1)
    v = p.mul_(support).sum(1, keepdim=True)
    tmp = (torch.sqrt(1 + 4 * 0.001 * (torch.abs(v) + 1 + 0.001)) - 1) / (2 * 0.001)
    return (torch.sign(v) * (tmp * tmp - 1)).float()


def run(B, S, secs, reference):
    model = bench.build_model(torch.device("cpu"), False, seed=0)
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32))
    support = torch.arange(-300, 301, dtype=torch.float64).unsqueeze(0)
    if reference:
        sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
        from gen_golden_ptree import load_reference_ptree
        pt, mmod = load_reference_ptree()
    random.seed(0)

    def recurrent(lat, acts, k):
        o = model.recurrent_inference(torch.from_numpy(np.asarray(lat)), torch.from_numpy(np.asarray(acts)).long())
        return (o.latent_state.numpy(), inverse(o.reward, support).numpy().reshape(-1).tolist(),
                inverse(o.value, support).numpy().reshape(-1).tolist(), o.policy_logits.numpy().tolist())

    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            out = model.initial_inference(obs)
            noises = rng.dirichlet([0.3, 0.3], size=B).astype(np.float32).tolist()
            legal = [[0, 1] for _ in range(B)]
            if reference:
                roots = pt.Roots(B, legal)
                roots.prepare(0.25, noises, [0.0] * B, out.policy_logits.numpy().tolist(), [-1] * B)
                pool = [out.latent_state.numpy()]
                mms = mmod.MinMaxStatsList(B)
                tp = [-1] * B
                for k in range(S):
                    res = pt.SearchResults(num=B)
                    x, y, acts, vtp = pt.batch_traverse(roots, 19652, 1.25, 0.997, mms, res, tp)
                    nxt, rew, val, lg = recurrent([pool[ix][iy] for ix, iy in zip(x, y)], acts, k)
                    pool.append(nxt)
                    pt.batch_backpropagate(k + 1, 0.997, rew, val, lg, mms, res, vtp)
                roots.get_distributions()
            else:
                roots = pp.PRoots(B, legal)
                roots.prepare(0.25, noises, [0.0] * B, out.policy_logits.numpy().tolist(), [-1] * B)
                pp.search(roots, recurrent, out.latent_state.numpy(), [-1] * B, S)
                roots.get_distributions()
            n += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return n * B * S / el, n, el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8)
    ap.add_argument("--sims", type=int, default=25)
    ap.add_argument("--secs", type=float, default=10.0)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--reference", action="store_true", help="the reference's own ptree (build container only)")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    v, n, el = run(a.envs, a.sims, a.secs, a.reference)
    print(json.dumps({"metric": "MCTS simulations/sec", "value": round(v, 1), "unit": "sims/s",
                      "config": {"workload": "C1 CartPole MuZero, pure-Python tree (ptree), MLP on CPU",
                                 "envs": a.envs, "num_simulations": a.sims},
                      "kind": "reference" if a.reference else "port", "cores": a.threads, "searches": n,
                      "seconds": round(el, 2), "host": bench.host_cpu_info()}))


if __name__ == "__main__":
    main()
