"""Generate the golden request/response transcripts under tests/golden/ (SURVEY.md §8(c)).

Test infrastructure only. This script drives the REFERENCE ctree (LightZero
``lzero/mcts/ctree/ctree_muzero/mz_tree.pyx`` and ``ctree_efficientzero/ez_tree.pyx``),
built from the sources under /root/reference by ``oracle/build_ref.sh`` into
``oracle/_ref/`` with ``gettimeofday`` wrapped so that the per-call
``srand(tv_usec)`` (``common_lib/utils.cpp:25``) takes a chosen seed.

The driving loop restates ``MuZeroMCTSCtree.search`` (``lzero/mcts/tree_search/mcts_ctree.py:228-321``)
and ``EfficientZeroMCTSCtree.search`` (``mcts_ctree.py:696-827``) with the network replaced by a
scripted table of responses, so each transcript holds, per simulation:
  requests  (x = latent_state_index_in_search_path, y = latent_state_index_in_batch,
             last_action, virtual_to_play, search_len)
  responses (reward | value_prefix, value, policy logits, and EZ is_reset)
and at the end the root visit distributions, root values and best-action trajectories.

Run (in the build container, where /root/reference exists):
    bash oracle/build_ref.sh && python tests/golden/gen_golden.py
The committed .npz files are data (inputs + expected outputs); the GPU box never needs
/root/reference.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")

PB_C_BASE = 19652
PB_C_INIT = 1.25
DISCOUNT = 0.997
VALUE_DELTA_MAX = 0.01
NOISE_WEIGHT = 0.25
ALPHA = 0.3
LSTM_HORIZON = 5


def traverse_seed(seed, k):
    """Per-traverse srand seed, SURVEY.md §8(d): usec_k = (1000003*seed + k) mod 1e6."""
    return (1000003 * seed + k) % 1000000


def make_case(name, tree, B, S, A, net, players, seed, noise=True, ragged=False):
    return dict(name=name, tree=tree, B=B, S=S, A=A, net=net, players=players, seed=seed,
                noise=noise, ragged=ragged)


CASES = [
    make_case("mz_zero_1p_b8_s25_a2", "mz", 8, 25, 2, "zero", 1, 0),
    make_case("mz_rand_1p_b8_s25_a2", "mz", 8, 25, 2, "rand", 1, 1),
    make_case("mz_zero_1p_b64_s25_a2", "mz", 64, 25, 2, "zero", 1, 2),
    make_case("mz_rand_1p_b64_s25_a2", "mz", 64, 25, 2, "rand", 1, 0),
    make_case("mz_zero_1p_b256_s50_a2", "mz", 256, 50, 2, "zero", 1, 1),
    make_case("mz_rand_1p_b256_s50_a2", "mz", 256, 50, 2, "rand", 1, 2),
    make_case("mz_quant_1p_b64_s50_a4", "mz", 64, 50, 4, "quant", 1, 0),
    make_case("mz_rand_1p_b32_s50_a6", "mz", 32, 50, 6, "rand", 1, 1),
    make_case("mz_zero_1p_b32_s50_a6", "mz", 32, 50, 6, "zero", 1, 2),
    make_case("mz_rand_1p_b32_s30_a4_nonoise", "mz", 32, 30, 4, "rand", 1, 0, noise=False),
    make_case("mz_rand_2p_b16_s50_a9", "mz", 16, 50, 9, "rand", 2, 1, ragged=True),
    make_case("mz_zero_2p_b16_s50_a9", "mz", 16, 50, 9, "zero", 2, 2, ragged=True),
    make_case("mz_quant_2p_b64_s25_a2", "mz", 64, 25, 2, "quant", 2, 0),
    make_case("mz_rand_1p_b48_s40_a5_ragged", "mz", 48, 40, 5, "rand", 1, 2, ragged=True),
    make_case("ez_rand_1p_b32_s50_a6", "ez", 32, 50, 6, "rand", 1, 0),
    make_case("ez_zero_1p_b32_s50_a6", "ez", 32, 50, 6, "zero", 1, 1),
    make_case("ez_quant_1p_b64_s50_a4", "ez", 64, 50, 4, "quant", 1, 2),
    make_case("ez_rand_2p_b16_s50_a9", "ez", 16, 50, 9, "rand", 2, 0, ragged=True),
]


def scripted(rng, net, shape):
    """Scripted network output tables (float32)."""
    if net == "zero":
        return np.zeros(shape, np.float32)
    if net == "rand":
        return rng.normal(0.0, 1.0, size=shape).astype(np.float32)
    if net == "quant":  # exact ties among visited children exercise the 1e-6 tie rule
        return rng.integers(-1, 2, size=shape).astype(np.float32)
    raise ValueError(net)


def gen_case(c, mods, lib):
    tree = mods[c["tree"]]
    B, S, A = c["B"], c["S"], c["A"]
    rng = np.random.default_rng(1000 + c["seed"] * 7 + B + S * 13 + A)
    # legal actions (ascending order, as the collector builds them from action_mask)
    legal_mask = np.ones((B, A), np.int8)
    if c["ragged"]:
        for i in range(B):
            k = int(rng.integers(1, A + 1))
            sel = np.sort(rng.choice(A, size=k, replace=False))
            legal_mask[i] = 0
            legal_mask[i, sel] = 1
    legal = [[a for a in range(A) if legal_mask[i, a]] for i in range(B)]
    if c["players"] == 1:
        to_play = [-1] * B
    else:
        to_play = [int(v) for v in rng.integers(1, 3, size=B)]
    noises = np.zeros((B, A), np.float32)
    for i in range(B):
        n = len(legal[i])
        noises[i, :n] = rng.dirichlet([ALPHA] * n).astype(np.float32)
    root_logits = scripted(rng, c["net"], (B, A))
    root_reward = np.zeros(B, np.float32) if c["tree"] == "mz" else scripted(rng, c["net"], (B,)) * 0.5

    resp_reward = scripted(rng, c["net"], (S, B)) * np.float32(0.5)
    resp_value = scripted(rng, c["net"], (S, B))
    resp_logits = scripted(rng, c["net"], (S, B, A))
    seeds = np.array([traverse_seed(c["seed"], k) for k in range(S)], np.int64)

    roots = tree.Roots(B, legal)
    if c["noise"]:
        roots.prepare(NOISE_WEIGHT, [noises[i, :len(legal[i])].tolist() for i in range(B)],
                      root_reward.tolist(), root_logits.tolist(), list(to_play))
    else:
        roots.prepare_no_noise(root_reward.tolist(), root_logits.tolist(), list(to_play))
    mms = tree.MinMaxStatsList(B)
    mms.set_delta(VALUE_DELTA_MAX)

    req = {k: np.zeros((S, B), np.int32) for k in ("x", "y", "a", "vtp", "len")}
    resp_reset = np.zeros((S, B), np.int32)
    for k in range(S):
        lib.oracle_set_usec(int(seeds[k]))
        res = tree.ResultsWrapper(num=B)
        x, y, a, vtp = tree.batch_traverse(roots, PB_C_BASE, PB_C_INIT, DISCOUNT, mms, res, list(to_play))
        slen = res.get_search_len()
        req["x"][k], req["y"][k], req["a"][k] = x, y, a
        req["vtp"][k], req["len"][k] = vtp, slen
        if c["tree"] == "mz":
            tree.batch_backpropagate(k + 1, DISCOUNT, resp_reward[k].tolist(), resp_value[k].tolist(),
                                     resp_logits[k].tolist(), mms, res, vtp)
        else:
            is_reset = (np.array(slen) % LSTM_HORIZON == 0).astype(np.int32)
            resp_reset[k] = is_reset
            tree.batch_backpropagate(k + 1, DISCOUNT, resp_reward[k].tolist(), resp_value[k].tolist(),
                                     resp_logits[k].tolist(), mms, res, is_reset.tolist(), vtp)
    dist = roots.get_distributions()
    out_dist = np.full((B, A), -1, np.int32)
    for i, d in enumerate(dist):
        out_dist[i, :len(d)] = d
    out_values = np.array(roots.get_values(), np.float32)
    trajs = roots.get_trajectories()
    tmax = max(1, max(len(t) for t in trajs))
    out_traj = np.full((B, tmax), -1, np.int32)
    for i, t in enumerate(trajs):
        out_traj[i, :len(t)] = t
    meta = np.array([B, S, A, c["players"], int(c["noise"]), 1 if c["tree"] == "ez" else 0, LSTM_HORIZON], np.int64)
    consts = np.array([PB_C_BASE, PB_C_INIT, DISCOUNT, VALUE_DELTA_MAX, NOISE_WEIGHT], np.float64)
    return dict(meta=meta, consts=consts, legal_mask=legal_mask, to_play=np.array(to_play, np.int32),
                noises=noises, root_logits=root_logits, root_reward=root_reward, seeds=seeds,
                req_x=req["x"], req_y=req["y"], req_a=req["a"], req_vtp=req["vtp"], req_len=req["len"],
                resp_reward=resp_reward, resp_value=resp_value, resp_logits=resp_logits,
                resp_is_reset=resp_reset, out_dist=out_dist, out_values=out_values, out_traj=out_traj)


def glibc_rand_vectors(lib_c):
    """Known-answer vectors of glibc srand/rand (the RNG cbatch_traverse uses, cnode.cpp:592)."""
    seeds = [0, 1, 12345, 999999, 2147483646]
    out = np.zeros((len(seeds), 2000), np.int64)
    for r, s in enumerate(seeds):
        lib_c.srand(ctypes.c_uint(s))
        for j in range(2000):
            out[r, j] = lib_c.rand()
    return np.array(seeds, np.int64), out


def main():
    if not os.path.isdir(REF_DIR):
        sys.exit("oracle/_ref missing: run oracle/build_ref.sh first")
    sys.path.insert(0, REF_DIR)
    import mz_tree  # noqa: E402  (reference build, test infrastructure)
    import ez_tree  # noqa: E402
    lib = ctypes.CDLL(mz_tree.__file__)
    lib.oracle_set_usec.argtypes = [ctypes.c_long]
    lib_ez = ctypes.CDLL(ez_tree.__file__)
    lib_ez.oracle_set_usec.argtypes = [ctypes.c_long]
    mods = {"mz": mz_tree, "ez": ez_tree}
    libs = {"mz": lib, "ez": lib_ez}
    for c in CASES:
        d = gen_case(c, mods, libs[c["tree"]])
        path = os.path.join(HERE, c["name"] + ".npz")
        np.savez_compressed(path, **d)
        lens = d["req_len"]
        print(f"{c['name']}: mean search_len {lens.mean():.2f} max {lens.max()} -> {os.path.basename(path)}")
    libc = ctypes.CDLL("libc.so.6")
    seeds, draws = glibc_rand_vectors(libc)
    np.savez_compressed(os.path.join(HERE, "glibc_rand.npz"), seeds=seeds, draws=draws)
    print("glibc_rand.npz written")


if __name__ == "__main__":
    main()
