"""GPU: ReZero search-with-reuse (mcts_ctree.py:323-420; mz_tree.pyx:84-107; cnode.cpp:502-546,
598-642, 702-749, 827-927).

1. The module API (lightzero_amd.ctree.mz_tree.batch_traverse_with_reuse /
   batch_backpropagate_with_reuse, driven exactly like the reference's loop with outputs compacted
   to the inferred envs) reproduces the reference's own transcripts (tests/golden/reuse_*.npz, made
   by tests/golden/gen_golden_reuse.py from the compiled reference): every request (x with -1 for
   skipped roots, y as the reference's compacted batch index, action, virtual_to_play, search_len),
   the final visit distributions, root values and trajectories — bit-exact.
2. MuZeroMCTSCtree.search_with_reuse on the device (one loop, reuse inputs on the tree handle)
   issues the same requests as that module API fed the values the kernels consumed, ends in the
   same tree, and returns the reference's (length, average_infer).
3. EfficientZero (reuse_ez_*; ez_tree.pyx:95-121, ctree_efficientzero/lib/cnode.cpp:603-641, 697-1073):
   the same two checks in the DEFINED form of the reference's EZ reuse search — is_reset passed
   per env (search_len % lstm_horizon_len == 0), since the reference loop's compacted list is read by
   env index (undefined once an env skips inference); the goldens come from the compiled reference
   tree called with that per-env list.
"""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
REUSE = sorted(glob.glob(os.path.join(GOLDEN, "reuse_*.npz")))
DEV = torch.device("cuda", 0)


class _Fixed:
    def __init__(self, v):
        self.v = int(v)

    def __call__(self):
        return self.v


def replay_module(tr, B, S, A, responses):
    """The reference's search_with_reuse loop over the module API; responses(k, inferred envs) ->
    (reward, value, logits) rows for those envs. Returns the requests and the final outputs."""
    from lightzero_amd.ctree import ez_tree, mz_tree
    from lightzero_amd.tree import set_seed_source
    ez = bool(int(tr["meta"][5])) if "meta" in tr else bool(tr.get("ez", False))
    horizon = int(tr["meta"][6]) if "meta" in tr else 5
    tree = ez_tree if ez else mz_tree
    legal = [[a for a in range(A) if tr["legal_mask"][i, a]] for i in range(B)]
    to_play = [int(v) for v in tr["to_play"]]
    roots = tree.Roots(B, legal)
    roots.prepare(float(tr["consts"][4]), [tr["noises"][i, :len(legal[i])].tolist() for i in range(B)], [0.0] * B,
                  tr["root_logits"].tolist(), list(to_play))
    mms = tree.MinMaxStatsList(B)
    mms.set_delta(float(tr["consts"][3]))
    ta, rv = [int(v) for v in tr["true_action"]], [float(v) for v in tr["reuse_value"]]
    got = {k: np.zeros((S, B), np.int64) for k in ("x", "y", "a", "vtp", "len")}
    for k in range(S):
        res = tree.ResultsWrapper(num=B)
        set_seed_source(_Fixed(tr["seeds"][k]))
        try:
            x, y, a, vtp = tree.batch_traverse_with_reuse(roots, 19652, 1.25, 0.997, mms, res, list(to_play), ta, rv)
        finally:
            set_seed_source(None)
        got["x"][k], got["y"][k], got["a"][k], got["vtp"][k] = x, y, a, vtp
        got["len"][k] = res.get_search_len()
        inf = [i for i in range(B) if x[i] != -1]
        no_inf = [i for i in range(B) if x[i] == -1] + [-1]
        reuse = [i for i in range(B) if x[i] == 0 and a[i] == ta[i]] + [-1]
        r, v, p = responses(k, inf)
        if ez:
            is_reset = [int(n % horizon == 0) for n in got["len"][k]]  # one flag per env (the defined form)
            tree.batch_backpropagate_with_reuse(k + 1, 0.997, r, v, p, mms, res, is_reset, vtp, no_inf, reuse, rv)
        else:
            tree.batch_backpropagate_with_reuse(k + 1, 0.997, r, v, p, mms, res, vtp, no_inf, reuse, rv)
    t = roots.tree
    got["dist"] = t.distributions().cpu().numpy()
    got["values"] = t.values().cpu().numpy()
    got["traj"] = t.trajectories(S + 2).cpu().numpy()
    roots.clear()
    return got


@pytest.mark.parametrize("path", REUSE, ids=lambda p: os.path.basename(p)[:-4])
def test_module_api_reproduces_reference_reuse_transcript(path):
    tr = dict(np.load(path))
    B, S, A = (int(v) for v in tr["meta"][:3])

    def responses(k, inf):
        return (tr["resp_reward"][k, inf].tolist(), tr["resp_value"][k, inf].tolist(),
                tr["resp_logits"][k, inf].tolist())
    got = replay_module(tr, B, S, A, responses)
    for key in ("x", "y", "a", "vtp", "len"):
        exp = tr["req_" + key]
        assert np.array_equal(got[key], exp), (key, np.argwhere(got[key] != exp)[:5])
    assert np.array_equal(got["dist"][:, :A], tr["out_dist"])
    assert np.array_equal(got["values"], tr["out_values"])
    tmax = tr["out_traj"].shape[1]
    assert np.array_equal(got["traj"][:, :tmax], tr["out_traj"])
    assert np.all(got["traj"][:, tmax:] == -1)


@pytest.mark.parametrize("quant,players", [(False, 1), (True, 1), (False, 2)])
def test_search_with_reuse_matches_module_api(quant, players):
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.utils import EasyDict
    from tests.helpers import NOISE_W, VDM, ScriptedTables, make_scripted_model
    B, S, A, seed = 48, 20, 3, 9
    tab = ScriptedTables(B, S, A, seed, players=players, quant=quant)
    rng = np.random.default_rng(seed)
    ta = rng.integers(0, A, size=B).astype(np.int32)
    rv = rng.normal(0, 1, size=B).astype(np.float32)
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, value_delta_max=float(VDM),
                        model=dict(support_scale=300, categorical_distribution=False)))
    mcts = MuZeroMCTSCtree(cfg)
    mcts.record = True
    roots = MuZeroMCTSCtree.roots(B, [list(range(A))] * B)
    roots.prepare(float(NOISE_W), [row.tolist() for row in tab.noises], [0.0] * B, tab.root_logits.tolist(),
                  tab.to_play.tolist())
    set_seed_source(SequentialSeeds(seed))
    try:
        length, avg = mcts.search_with_reuse(roots, make_scripted_model(tab, DEV), tab.lat0, tab.to_play.tolist(),
                                             ta.tolist(), rv.tolist())
    finally:
        set_seed_source(None)
    rec = mcts.last_record.numpy()
    t = roots.tree
    dev_out = dict(dist=t.distributions().cpu().numpy(), values=t.values().cpu().numpy(),
                   traj=t.trajectories(S + 2).cpu().numpy())
    roots.clear()
    inferred = (rec["x"] != -1).sum(axis=1)
    assert length == int(inferred[-1]) and avg == pytest.approx(inferred.sum() / S)
    assert (rec["x"] == -1).any(), "the case exercises no skipped inference"
    # the module API fed the values the device loop consumed
    tr = dict(legal_mask=np.ones((B, A), np.int8), to_play=tab.to_play, noises=tab.noises,
              root_logits=tab.root_logits, consts=np.array([19652, 1.25, 0.997, VDM, NOISE_W], np.float64),
              true_action=ta, reuse_value=rv, seeds=np.asarray(rec["seeds"]).astype(np.int64))

    def responses(k, inf):
        return (rec["decoded"][k][inf, 0].tolist(), rec["decoded"][k][inf, 1].tolist(),
                rec["policy_logits"][k][inf].tolist())
    got = replay_module(tr, B, S, A, responses)
    for key, rk in (("x", "x"), ("a", "action"), ("len", "search_len")):
        assert np.array_equal(got[key], rec[rk]), key
    for key in ("dist", "values", "traj"):
        assert np.array_equal(got[key], dev_out[key]), key


def make_scripted_ez_model(tab, device, Hl=4):
    """ScriptedTables behind the EfficientZero recurrent_inference surface (value prefix, LSTM state)."""
    class Out:
        pass

    class ScriptedEZ(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.k = 0
            self.r = torch.from_numpy(tab.r).to(device)
            self.v = torch.from_numpy(tab.v).to(device)
            self.p = torch.from_numpy(tab.p).to(device)

        def recurrent_inference(self, latent, hidden, action):
            k = self.k
            self.k += 1
            s = latent.sum(dim=1)
            o = Out()
            o.value_prefix = (self.r[k] + 0.01 * s).unsqueeze(1)
            o.value = (self.v[k] + 0.01 * s).unsqueeze(1)
            o.policy_logits = self.p[k] + 0.01 * latent[:, :1]
            o.latent_state = latent + (action.to(torch.float32) + 1.0).unsqueeze(1)
            o.reward_hidden_state = (hidden[0] + 1.0, hidden[1] + 2.0)
            return o

    return ScriptedEZ()


@pytest.mark.parametrize("quant,players", [(False, 1), (True, 1), (False, 2)])
def test_ez_search_with_reuse_matches_module_api(quant, players):
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.utils import EasyDict
    from tests.helpers import NOISE_W, VDM, ScriptedTables
    B, S, A, seed, Hl = 48, 20, 3, 11, 4
    tab = ScriptedTables(B, S, A, seed, players=players, quant=quant)
    rng = np.random.default_rng(seed)
    ta = rng.integers(0, A, size=B).astype(np.int32)
    rv = rng.normal(0, 1, size=B).astype(np.float32)
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, value_delta_max=float(VDM),
                        lstm_horizon_len=5, model=dict(support_scale=300, categorical_distribution=False)))
    mcts = EfficientZeroMCTSCtree(cfg)
    mcts.record = True
    roots = EfficientZeroMCTSCtree.roots(B, [list(range(A))] * B)
    roots.prepare(float(NOISE_W), [row.tolist() for row in tab.noises], [0.0] * B, tab.root_logits.tolist(),
                  tab.to_play.tolist())
    h0 = torch.zeros(1, B, Hl, device=DEV)
    set_seed_source(SequentialSeeds(seed))
    try:
        length, avg = mcts.search_with_reuse(roots, make_scripted_ez_model(tab, DEV, Hl), tab.lat0, (h0, h0),
                                             tab.to_play.tolist(), ta.tolist(), rv.tolist())
    finally:
        set_seed_source(None)
    rec = mcts.last_record.numpy()
    is_reset = mcts.last_record.is_reset.cpu().numpy()
    t = roots.tree
    dev_out = dict(dist=t.distributions().cpu().numpy(), values=t.values().cpu().numpy(),
                   traj=t.trajectories(S + 2).cpu().numpy())
    roots.clear()
    inferred = (rec["x"] != -1).sum(axis=1)
    assert length == int(inferred[-1]) and avg == pytest.approx(inferred.sum() / S)
    assert (rec["x"] == -1).any(), "the case exercises no skipped inference"
    assert np.array_equal(is_reset, (rec["search_len"] % 5 == 0).astype(np.int32))  # per env, every env
    tr = dict(legal_mask=np.ones((B, A), np.int8), to_play=tab.to_play, noises=tab.noises,
              root_logits=tab.root_logits, consts=np.array([19652, 1.25, 0.997, VDM, NOISE_W], np.float64),
              true_action=ta, reuse_value=rv, seeds=np.asarray(rec["seeds"]).astype(np.int64),
              meta=np.array([B, S, A, players, 1, 1, 5], np.int64))

    def responses(k, inf):
        return (rec["decoded"][k][inf, 0].tolist(), rec["decoded"][k][inf, 1].tolist(),
                rec["policy_logits"][k][inf].tolist())
    got = replay_module(tr, B, S, A, responses)
    for key, rk in (("x", "x"), ("a", "action"), ("len", "search_len")):
        assert np.array_equal(got[key], rec[rk]), key
    for key in ("dist", "values", "traj"):
        assert np.array_equal(got[key], dev_out[key]), key


def test_ez_reuse_rejects_the_compacted_is_reset_list():
    """the reference loop's is_reset_list over the inferred envs only is refused (its by-env read is
    undefined once an env skips inference)"""
    from lightzero_amd.ctree import ez_tree
    from lightzero_amd.tree import set_seed_source
    B, A = 8, 2
    roots = ez_tree.Roots(B, [[0, 1]] * B)
    roots.prepare(0.25, [[0.5, 0.5]] * B, [0.0] * B, [[1.0, 0.0]] * B, [-1] * B)
    mms = ez_tree.MinMaxStatsList(B)
    res = ez_tree.ResultsWrapper(num=B)
    set_seed_source(_Fixed(7))
    try:
        x, y, a, vtp = ez_tree.batch_traverse_with_reuse(roots, 19652, 1.25, 0.997, mms, res, [-1] * B, [0] * B,
                                                         [0.5] * B)
    finally:
        set_seed_source(None)
    with pytest.raises(ValueError, match="one flag per env"):
        ez_tree.batch_backpropagate_with_reuse(1, 0.997, [0.0] * B, [0.0] * B, [[0.0, 0.0]] * B, mms, res, [0] * (B - 1),
                                               vtp, [-1], [-1], [0.5] * B)
    roots.clear()
