"""CPU: the oracle (oracle/lz_oracle.c, a restatement of the reference ctree) pinned against the
golden transcripts recorded from the reference build (tests/golden/gen_golden.py)."""
import glob
import os

import numpy as np
import pytest

from oracle.oracle import (OracleTree, glibc_rand_stream, lib, load_transcript, philox4x32_10,
                           replay_transcript)
from tests.helpers import random_transcript, run_scripted_search_oracle, run_transcript

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TRANSCRIPTS = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz")) if not p.endswith("glibc_rand.npz") and not os.path.basename(p).startswith(("az_", "reuse_", "ptree_")))


def test_golden_files_present():
    assert len(TRANSCRIPTS) >= 18


@pytest.mark.parametrize("path", TRANSCRIPTS, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_reference_transcript(path):
    bad = replay_transcript(load_transcript(path))
    assert not bad, bad


def test_glibc_rand_restatement_matches_libc_vectors():
    g = np.load(os.path.join(GOLDEN, "glibc_rand.npz"))
    for seed, draws in zip(g["seeds"], g["draws"]):
        assert np.array_equal(glibc_rand_stream(int(seed), draws.shape[0]), draws), seed


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10
    assert philox4x32_10([0, 0, 0, 0], [0, 0]).tolist() == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert philox4x32_10([0xffffffff] * 4, [0xffffffff] * 2).tolist() == [0x408f276d, 0x41c83b0e, 0xa20bc7c6,
                                                                            0x6d5451fd]
    assert philox4x32_10([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]).tolist() == [
        0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


@pytest.mark.parametrize("fast", [False, True])
def test_oracle_visit_counts_conserved(fast):
    B, S, A = 32, 30, 4
    out = run_transcript(random_transcript(B, S, A, seed=3), OracleTree, fast_rng=fast)
    # every simulation adds exactly one visit below the root
    assert (out["dist"].sum(axis=1) == S).all()
    assert (out["len"] >= 1).all()


def test_oracle_fast_mode_independent_of_batch_composition():
    # Philox draws depend on (seed, root, level) only: the first 8 roots of a 32-root batch
    # search exactly like an 8-root batch (not true of the serial glibc stream).
    tr32 = random_transcript(32, 20, 3, seed=5, net="quant")
    tr8 = {k: (v[:8] if k in ("legal_mask", "to_play", "noises", "root_logits", "root_reward") else v)
           for k, v in tr32.items()}
    tr8["meta"] = tr32["meta"].copy()
    tr8["meta"][0] = 8
    for k in ("resp_reward", "resp_value", "resp_is_reset"):
        tr8[k] = tr32[k][:, :8]
    tr8["resp_logits"] = tr32["resp_logits"][:, :8]
    a = run_transcript(tr32, OracleTree, fast_rng=True)
    b = run_transcript(tr8, OracleTree, fast_rng=True)
    assert np.array_equal(a["dist"][:8], b["dist"])


def test_host_search_loop_is_deterministic():
    a = run_scripted_search_oracle(16, 20, 3, seed=1)
    b = run_scripted_search_oracle(16, 20, 3, seed=1)
    assert np.array_equal(a["dist"], b["dist"]) and np.array_equal(a["values"], b["values"])
    assert (a["dist"].sum(axis=1) == 20).all()


def test_cpu_baseline_driver_runs():
    secs = lib().lzo_bench_tree_only(64, 2, 10, 2, 1, 1)
    assert secs > 0


def test_path_scores_diagnostic_agrees_with_traverse():
    """oracle.path_scores (the divergence attribution's tool): along every root's traverse path the
    action taken is in the tie list of the scores the diagnostic recomputes at that level"""
    from tests.helpers import tie_list
    tr = random_transcript(24, 16, 3, seed=9, net="rand")
    B, S, A = 24, 16, 3
    ot = OracleTree(B, A, S)
    ot.set_delta(np.float32(0.01))
    ot.prepare(np.float32(0.25), tr["noises"], tr["root_reward"], tr["root_logits"], np.full(B, -1, np.int32))
    levels = 0
    for k in range(S):
        x, y, a, vtp, slen = ot.traverse(19652, np.float32(1.25), np.float32(0.997), 1000 + k, np.full(B, -1, np.int32))
        for i in range(B):
            acts = ot.path_actions(i)
            assert len(acts) == slen[i] and acts[-1] == a[i]
            sc = ot.path_scores(i, acts)
            assert sc.shape[0] == len(acts)  # the leaf below the last action is not expanded yet
            for lvl, act in enumerate(acts):
                assert act in tie_list(sc[lvl]), (k, i, lvl)
                levels += 1
        ot.backprop(k + 1, np.float32(0.997), tr["resp_reward"][k], tr["resp_value"][k], tr["resp_logits"][k], vtp)
    assert levels > B * S
