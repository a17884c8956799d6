"""Generate tests/golden/ptree_*.npz: transcripts of the REFERENCE pure-Python MuZero tree (config 1).

Test infrastructure only. Loads /root/reference/lzero/mcts/ptree/ptree_mz.py (and the minimax.py it
imports) by file path — an alias package pointing at that directory, so lzero/__init__.py and
DI-engine are never imported — and drives its Roots / batch_traverse / batch_backpropagate with the
loop of MuZeroMCTSPtree.search (lzero/mcts/tree_search/mcts_ptree.py:92-194) restated here, the
network replaced by a scripted table of decoded outputs, and Python's global `random` seeded (the
reference breaks ties with random.choice, ptree_mz.py:366). Each transcript holds the inputs (legal
sets, noises, root logits, the per-simulation rewards / values / logits) and the expected outputs
(per-simulation requests, final visit distributions, root values, trajectories). oracle/ptree_port.py
must reproduce them exactly (tests/test_ptree_port.py).

Run in the build container (where /root/reference exists):  python tests/golden/gen_golden_ptree.py
"""
import importlib
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PTREE_DIR = "/root/reference/lzero/mcts/ptree"
PB_C_BASE, PB_C_INIT, DISC, NOISE_W = 19652, 1.25, 0.997, 0.25

CASES = [  # name, B, S, A, net, seed, ragged legal sets
    ("ptree_rand_b8_s25_a2", 8, 25, 2, "rand", 0, False),
    ("ptree_rand_b8_s25_a2_s1", 8, 25, 2, "rand", 1, False),
    ("ptree_zero_b8_s25_a2", 8, 25, 2, "zero", 2, False),
    ("ptree_rand_b16_s30_a4_ragged", 16, 30, 4, "rand", 3, True),
]


def load_reference_ptree():
    pkg = types.ModuleType("ref_ptree")
    pkg.__path__ = [PTREE_DIR]
    sys.modules["ref_ptree"] = pkg
    return importlib.import_module("ref_ptree.ptree_mz"), importlib.import_module("ref_ptree.minimax")


def scripted(B, S, A, net, seed):
    g = np.random.default_rng(1000 + seed)
    if net == "zero":
        return (np.zeros((S, B), np.float32), np.zeros((S, B), np.float32), np.zeros((S, B, A), np.float32))
    return ((g.standard_normal((S, B)) * 0.5).astype(np.float32), g.standard_normal((S, B)).astype(np.float32),
            g.standard_normal((S, B, A)).astype(np.float32))


def gen_case(pt, mmod, name, B, S, A, net, seed, ragged):
    g = np.random.default_rng(seed)
    if ragged:
        legal = [sorted(g.choice(A, size=int(g.integers(1, A + 1)), replace=False).tolist()) for _ in range(B)]
    else:
        legal = [list(range(A)) for _ in range(B)]
    noises = [g.dirichlet([0.3] * len(l)).astype(np.float32).tolist() for l in legal]
    logits0 = g.standard_normal((B, A)).astype(np.float32)
    rew, val, lg = scripted(B, S, A, net, seed)
    roots = pt.Roots(B, legal)
    roots.prepare(NOISE_W, noises, [0.0] * B, logits0.tolist(), [-1] * B)
    random.seed(seed)
    mms = mmod.MinMaxStatsList(B)
    to_play = [-1] * B
    rec = {k: np.zeros((S, B), np.int64) for k in ("x", "y", "action", "search_len")}
    for k in range(S):
        res = pt.SearchResults(num=B)
        x, y, acts, vtp = pt.batch_traverse(roots, PB_C_BASE, PB_C_INIT, DISC, mms, res, to_play)
        rec["x"][k], rec["y"][k], rec["action"][k], rec["search_len"][k] = x, y, acts, res.search_lens
        pt.batch_backpropagate(k + 1, DISC, rew[k].tolist(), val[k].tolist(), lg[k].tolist(), mms, res, vtp)
    dist = roots.get_distributions()
    trajs = roots.get_trajectories()
    T = S + 2
    dist_arr = np.full((B, A), -1, np.int64)
    for i, d in enumerate(dist):
        dist_arr[i, :len(d)] = d
    traj_arr = np.full((B, T), -1, np.int64)
    for i, t in enumerate(trajs):
        traj_arr[i, :len(t)] = t
    legal_arr = np.full((B, A), -1, np.int64)
    for i, l in enumerate(legal):
        legal_arr[i, :len(l)] = l
    noise_arr = np.zeros((B, A), np.float32)
    for i, n in enumerate(noises):
        noise_arr[i, :len(n)] = n
    np.savez_compressed(os.path.join(HERE, name + ".npz"), B=B, S=S, A=A, seed=seed, legal=legal_arr,
                        noises=noise_arr, logits0=logits0, rewards=rew, values=val, logits=lg, x=rec["x"],
                        y=rec["y"], action=rec["action"], search_len=rec["search_len"], dist=dist_arr,
                        root_values=np.array(roots.get_values(), np.float64), traj=traj_arr)
    print(name, "dist row 0:", dist[0], "value 0:", roots.get_values()[0])


def main():
    pt, mmod = load_reference_ptree()
    for c in CASES:
        gen_case(pt, mmod, *c)


if __name__ == "__main__":
    main()
