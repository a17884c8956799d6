"""GPU: the HIP tree (traverse / backprop through the C ABI) against the reference's golden
transcripts and, at sizes beyond the fixtures, against the oracle on identical inputs.
Bit-exact: every request (x, y, action, virtual_to_play, search_len) of every simulation, the
final visit distributions, root values and best-action trajectories."""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle.oracle import OracleTree, load_transcript, replay_transcript  # noqa: E402
from tests.helpers import GpuTree, random_transcript, run_transcript  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TRANSCRIPTS = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz")) if not p.endswith("glibc_rand.npz") and not os.path.basename(p).startswith(("az_", "reuse_", "ptree_")))


@pytest.mark.parametrize("path", TRANSCRIPTS, ids=lambda p: os.path.basename(p)[:-4])
def test_gpu_reproduces_reference_transcript(path):
    bad = replay_transcript(load_transcript(path), tree_factory=GpuTree)
    assert not bad, bad


def assert_same(a, b):
    for k in ("x", "y", "a", "vtp", "len", "dist", "traj"):
        if not np.array_equal(a[k], b[k]):
            idx = np.argwhere(a[k] != b[k])[:5]
            raise AssertionError(f"{k} differs at {idx.tolist()}")
    assert np.array_equal(a["values"], b["values"]), np.abs(a["values"] - b["values"]).max()


CASES = [
    # (B, S, A, players, ez, net, ragged)
    (256, 50, 2, 1, False, "rand", False),
    (256, 50, 2, 1, False, "zero", False),
    (256, 50, 2, 2, False, "quant", False),
    (512, 100, 9, 2, False, "rand", True),
    (1024, 50, 4, 1, False, "quant", False),
    (2048, 30, 4, 1, False, "rand", False),  # > one workgroup of roots per traverse round
    (1, 20, 1, 1, False, "rand", False),
    (3, 15, 64, 1, False, "rand", True),
    (100, 40, 6, 1, True, "rand", False),
    (64, 50, 18, 2, True, "quant", True),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b{}_s{}_a{}_p{}_{}_{}{}".format(
    c[0], c[1], c[2], c[3], "ez" if c[4] else "mz", c[5], "_ragged" if c[6] else ""))
def test_gpu_matches_oracle_parity_mode(case):
    B, S, A, players, ez, net, ragged = case
    tr = random_transcript(B, S, A, seed=B + S + A, players=players, ez=ez, net=net, ragged=ragged)
    assert_same(run_transcript(tr, GpuTree), run_transcript(tr, OracleTree))


# parity mode runs one wave per root with a decoupled look-back of the draw offsets
# (lzm_traverse_lb.h); LZM_TRAVERSE=serial keeps the one-workgroup fixed-point kernel
@pytest.mark.parametrize("case", [CASES[1], CASES[3], CASES[5], CASES[9]], ids=lambda c: f"b{c[0]}_a{c[2]}_{c[5]}")
def test_serial_traverse_kernel_matches_oracle(case, monkeypatch):
    monkeypatch.setenv("LZM_TRAVERSE", "serial")
    test_gpu_matches_oracle_parity_mode(case)


@pytest.mark.parametrize("case", [(256, 50, 2, 1, False), (512, 30, 9, 2, False), (128, 40, 6, 1, True)])
def test_gpu_matches_oracle_fast_mode(case):
    B, S, A, players, ez = case
    tr = random_transcript(B, S, A, seed=7 * B + S, players=players, ez=ez, net="quant")
    assert_same(run_transcript(tr, GpuTree, fast_rng=True), run_transcript(tr, OracleTree, fast_rng=True))


def test_empty_legal_list_means_all_actions():
    # CNode::expand fills 0..A-1 when legal_actions is empty (cnode.cpp:101-107)
    tr = random_transcript(8, 10, 3, seed=1)
    B, A = 8, 3
    gt = GpuTree(B, A, 10)
    ot = OracleTree(B, A, 10)
    legal = np.full((B, A), -1, np.int32)
    cnt = np.zeros(B, np.int32)
    gt.set_legal(legal, cnt)
    full = np.tile(np.arange(A, dtype=np.int32), (B, 1))
    ot.set_legal(full, np.full(B, A, np.int32))
    for t in (gt, ot):
        t.set_delta(np.float32(0.01))
        t.prepare(np.float32(0.25), tr["noises"][:, :A], tr["root_reward"], tr["root_logits"], tr["to_play"])
    for k in range(10):
        og = gt.traverse(19652, np.float32(1.25), np.float32(0.997), k + 11, tr["to_play"])
        oo = ot.traverse(19652, np.float32(1.25), np.float32(0.997), k + 11, tr["to_play"])
        assert all(np.array_equal(a, b) for a, b in zip(og, oo))
        for t, o in ((gt, og), (ot, oo)):
            t.backprop(k + 1, np.float32(0.997), tr["resp_reward"][k], tr["resp_value"][k], tr["resp_logits"][k], o[3])
    assert np.array_equal(gt.distributions(), ot.distributions())


def test_module_api_matches_oracle_and_grows_capacity():
    """mz_tree-compatible list API (mz_tree.pyx surface); 80 simulations > default capacity."""
    from lightzero_amd.ctree import mz_tree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    B, S, A = 40, 80, 3
    tr = random_transcript(B, S, A, seed=99)
    roots = mz_tree.Roots(B, [list(range(A)) for _ in range(B)])
    roots.prepare(0.25, [r.tolist() for r in tr["noises"]], [0.0] * B, tr["root_logits"].tolist(), [-1] * B)
    mms = mz_tree.MinMaxStatsList(B)
    mms.set_delta(0.01)
    ot = OracleTree(B, A, S)
    ot.set_delta(np.float32(0.01))
    ot.prepare(np.float32(0.25), tr["noises"], np.zeros(B, np.float32), tr["root_logits"], np.full(B, -1, np.int32))
    set_seed_source(SequentialSeeds(99))
    try:
        for k in range(S):
            res = mz_tree.ResultsWrapper(num=B)
            x, y, a, vtp = mz_tree.batch_traverse(roots, 19652, 1.25, 0.997, mms, res, [-1] * B)
            ox, oy, oa, ovtp, olen = ot.traverse(19652, np.float32(1.25), np.float32(0.997),
                                                 (1000003 * 99 + k) % 1000000, np.full(B, -1, np.int32))
            assert x == ox.tolist() and y == oy.tolist() and a == oa.tolist() and vtp == ovtp.tolist()
            assert res.get_search_len() == olen.tolist()
            mz_tree.batch_backpropagate(k + 1, 0.997, tr["resp_reward"][k % tr["resp_reward"].shape[0]].tolist(),
                                        tr["resp_value"][k].tolist(), tr["resp_logits"][k].tolist(), mms, res, vtp)
            ot.backprop(k + 1, np.float32(0.997), tr["resp_reward"][k], tr["resp_value"][k], tr["resp_logits"][k],
                        ovtp)
    finally:
        set_seed_source(None)
    assert roots.get_distributions() == [[int(v) for v in row] for row in ot.distributions()]
    assert np.array_equal(np.array(roots.get_values(), np.float32), ot.values())
    traj = ot.trajectories(S + 2)
    assert roots.get_trajectories() == [[int(v) for v in row if v >= 0] for row in traj]


def test_traverse_passes_small():
    """Parity mode settles the batch-serial rand() offsets in few speculative passes."""
    B, S, A = 256, 30, 2
    tr = random_transcript(B, S, A, seed=5)
    gt = GpuTree(B, A, S)
    from oracle.oracle import legal_from_mask
    legal, cnt = legal_from_mask(tr["legal_mask"])
    gt.set_legal(legal, cnt)
    gt.set_delta(np.float32(0.01))
    gt.prepare(np.float32(0.25), tr["noises"], tr["root_reward"], tr["root_logits"], tr["to_play"])
    passes = []
    for k in range(S):
        o = gt.traverse(19652, np.float32(1.25), np.float32(0.997), int(tr["seeds"][k]), tr["to_play"])
        passes.append(gt.t.traverse_passes())
        gt.backprop(k + 1, np.float32(0.997), tr["resp_reward"][k], tr["resp_value"][k], tr["resp_logits"][k], o[3])
    gt.t.check_errors()  # raises on a look-back timeout / draw-table overflow (sticky err words)
    assert max(p[0] for p in passes) <= 4, passes
