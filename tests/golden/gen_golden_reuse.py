"""Golden transcripts of the reference's ReZero search-with-reuse (test infrastructure only).

Drives the REFERENCE ctree built by ``oracle/build_ref.sh`` into ``oracle/_ref/`` (``mz_tree``:
``batch_traverse_with_reuse`` / ``batch_backpropagate_with_reuse``, ``mz_tree.pyx:84-107``,
``ctree_muzero/lib/cnode.cpp:502-546, 598-642, 702-749, 827-927``) with the loop of
``MuZeroMCTSCtree.search_with_reuse`` (``lzero/mcts/tree_search/mcts_ctree.py:323-420``) and the
network replaced by scripted per-env tables: envs whose walk ends on an expanded node (the root
child of the true action) get no inference (x = -1) and back up their reuse value; envs stopping
at the unexpanded true-action child are expanded but back up the reuse value too. The reference
consumes the outputs compacted to the inferred envs; the transcript stores the full tables.

EfficientZero cases (``reuse_ez_*``) drive ``ez_tree`` (``ez_tree.pyx:95-121``,
``ctree_efficientzero/lib/cnode.cpp:603-641, 697-1073``) with the loop of
``EfficientZeroMCTSCtree.search_with_reuse`` (``mcts_ctree.py:829-955``) in its DEFINED form: the
reference loop builds ``is_reset_list`` over the inferred envs only, while the tree reads it by env
index (an out-of-range read once an env skips inference), so here the list holds one flag per env,
``search_len % lstm_horizon_len == 0`` — what the reference passes when no env skips. The tree
call itself is the reference's, unchanged.

    bash oracle/build_ref.sh && python tests/golden/gen_golden_reuse.py
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import (ALPHA, DISCOUNT, LSTM_HORIZON, NOISE_WEIGHT, PB_C_BASE, PB_C_INIT, REF_DIR,  # noqa: E402
                        VALUE_DELTA_MAX, scripted, traverse_seed)

CASES = [
    dict(name="reuse_rand_1p_b32_s30_a4", B=32, S=30, A=4, net="rand", players=1, seed=3, ragged=False),
    dict(name="reuse_quant_1p_b64_s25_a2", B=64, S=25, A=2, net="quant", players=1, seed=4, ragged=False),
    dict(name="reuse_rand_2p_b16_s30_a5", B=16, S=30, A=5, net="rand", players=2, seed=5, ragged=True),
    dict(name="reuse_zero_1p_b16_s20_a3", B=16, S=20, A=3, net="zero", players=1, seed=6, ragged=False),
    dict(name="reuse_ez_rand_1p_b32_s30_a4", B=32, S=30, A=4, net="rand", players=1, seed=7, ragged=False, ez=True),
    dict(name="reuse_ez_quant_1p_b48_s25_a3", B=48, S=25, A=3, net="quant", players=1, seed=8, ragged=True, ez=True),
    dict(name="reuse_ez_rand_2p_b16_s30_a5", B=16, S=30, A=5, net="rand", players=2, seed=9, ragged=True, ez=True),
]


def gen_case(c, tree, lib):
    B, S, A = c["B"], c["S"], c["A"]
    rng = np.random.default_rng(5000 + c["seed"] * 11 + B + S * 7 + A)
    legal_mask = np.ones((B, A), np.int8)
    if c["ragged"]:
        for i in range(B):
            k = int(rng.integers(1, A + 1))
            sel = np.sort(rng.choice(A, size=k, replace=False))
            legal_mask[i] = 0
            legal_mask[i, sel] = 1
    legal = [[a for a in range(A) if legal_mask[i, a]] for i in range(B)]
    to_play = [-1] * B if c["players"] == 1 else [int(v) for v in rng.integers(1, 3, size=B)]
    noises = np.zeros((B, A), np.float32)
    for i in range(B):
        noises[i, :len(legal[i])] = rng.dirichlet([ALPHA] * len(legal[i])).astype(np.float32)
    true_action = np.array([legal[i][int(rng.integers(0, len(legal[i])))] for i in range(B)], np.int32)
    reuse_value = (rng.normal(0.0, 1.0, size=B) if c["net"] != "zero" else np.zeros(B)).astype(np.float32)
    root_logits = scripted(rng, c["net"], (B, A))
    resp_reward = scripted(rng, c["net"], (S, B)) * np.float32(0.5)
    resp_value = scripted(rng, c["net"], (S, B))
    resp_logits = scripted(rng, c["net"], (S, B, A))
    seeds = np.array([traverse_seed(c["seed"], k) for k in range(S)], np.int64)
    roots = tree.Roots(B, legal)
    roots.prepare(NOISE_WEIGHT, [noises[i, :len(legal[i])].tolist() for i in range(B)], [0.0] * B,
                  root_logits.tolist(), list(to_play))
    mms = tree.MinMaxStatsList(B)
    mms.set_delta(VALUE_DELTA_MAX)
    req = {k: np.zeros((S, B), np.int32) for k in ("x", "y", "a", "vtp", "len")}
    is_reset = np.zeros((S, B), np.int32)
    infer = np.zeros(S, np.int64)
    for k in range(S):
        lib.oracle_set_usec(int(seeds[k]))
        res = tree.ResultsWrapper(num=B)
        x, y, a, vtp = tree.batch_traverse_with_reuse(roots, PB_C_BASE, PB_C_INIT, DISCOUNT, mms, res, list(to_play),
                                                      true_action.tolist(), reuse_value.tolist())
        req["x"][k], req["y"][k], req["a"][k], req["vtp"][k] = x, y, a, vtp
        req["len"][k] = res.get_search_len()
        inf = [i for i in range(B) if x[i] != -1]
        no_inf = [i for i in range(B) if x[i] == -1] + [-1]
        reuse = [i for i in range(B) if x[i] == 0 and a[i] == true_action[i]] + [-1]
        infer[k] = len(inf)
        if c.get("ez"):
            is_reset[k] = (req["len"][k] % LSTM_HORIZON == 0).astype(np.int32)  # one flag per env
            tree.batch_backpropagate_with_reuse(k + 1, DISCOUNT, resp_reward[k, inf].tolist(),
                                                resp_value[k, inf].tolist(), resp_logits[k, inf].tolist(), mms, res,
                                                is_reset[k].tolist(), vtp, no_inf, reuse, reuse_value.tolist())
        else:
            tree.batch_backpropagate_with_reuse(k + 1, DISCOUNT, resp_reward[k, inf].tolist(),
                                                resp_value[k, inf].tolist(), resp_logits[k, inf].tolist(), mms, res,
                                                vtp, no_inf, reuse, reuse_value.tolist())
    dist = roots.get_distributions()
    out_dist = np.full((B, A), -1, np.int32)
    for i, d in enumerate(dist):
        out_dist[i, :len(d)] = d
    trajs = roots.get_trajectories()
    tmax = max(1, max(len(t) for t in trajs))
    out_traj = np.full((B, tmax), -1, np.int32)
    for i, t in enumerate(trajs):
        out_traj[i, :len(t)] = t
    meta = np.array([B, S, A, c["players"], 1, 1 if c.get("ez") else 0, LSTM_HORIZON if c.get("ez") else 0], np.int64)
    consts = np.array([PB_C_BASE, PB_C_INIT, DISCOUNT, VALUE_DELTA_MAX, NOISE_WEIGHT], np.float64)
    return dict(meta=meta, consts=consts, legal_mask=legal_mask, to_play=np.array(to_play, np.int32), noises=noises,
                root_logits=root_logits, root_reward=np.zeros(B, np.float32), seeds=seeds,
                true_action=true_action, reuse_value=reuse_value, req_x=req["x"], req_y=req["y"], req_a=req["a"],
                req_vtp=req["vtp"], req_len=req["len"], infer=infer, resp_reward=resp_reward,
                resp_value=resp_value, resp_logits=resp_logits, is_reset=is_reset, out_dist=out_dist,
                out_values=np.array(roots.get_values(), np.float32), out_traj=out_traj)


def main():
    if not os.path.isdir(REF_DIR):
        sys.exit("oracle/_ref missing: run oracle/build_ref.sh first")
    sys.path.insert(0, REF_DIR)
    import ez_tree  # noqa: E402  (reference build, test infrastructure)
    import mz_tree  # noqa: E402
    libs = {}
    for name, mod in (("mz", mz_tree), ("ez", ez_tree)):
        libs[name] = ctypes.CDLL(mod.__file__)
        libs[name].oracle_set_usec.argtypes = [ctypes.c_long]
    for c in CASES:
        kind = "ez" if c.get("ez") else "mz"
        d = gen_case(c, ez_tree if kind == "ez" else mz_tree, libs[kind])
        np.savez_compressed(os.path.join(HERE, c["name"] + ".npz"), **d)
        x = d["req_x"]
        print(f"{c['name']}: no-inference {(x == -1).mean():.3f}, reuse-expanded "
              f"{((x == 0) & (d['req_a'] == d['true_action'][None])).mean():.3f}, mean len {d['req_len'].mean():.2f}")


if __name__ == "__main__":
    main()
