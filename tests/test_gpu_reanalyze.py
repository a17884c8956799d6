"""GPU: reanalyze-sized searches (B = batch x (K+1) = 1,536 roots).

1. The fused search at B = 1,536 (8 roots per workgroup, 192 workgroups) is bit-exact with the
   oracle fed the recorded network outputs (as tests/test_gpu_fused.py does at B <= 256).
2. reanalyze_policy_targets = normalised root visit counts scattered onto the legal actions of
   each position (ragged legal sets), zeros where policy_mask is 0 — compared with the same search
   run through MuZeroMCTSCtree directly.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def test_fused_search_reanalyze_batch_exact():
    from tests.test_gpu_fused import check_tree_exact
    check_tree_exact((1536, 50, 2, 128, False, 1, False))


def test_reanalyze_policy_targets():
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.reanalyze import reanalyze_policy_targets
    from lightzero_amd.utils import EasyDict
    from tests.test_gpu_fused import make_model
    N, A, S = 384, 3, 20
    model = make_model(A, 64, False, seed=4)
    rng = np.random.default_rng(1)
    obs = torch.from_numpy(rng.normal(size=(N, 4)).astype(np.float32)).to(DEV)
    mask = np.ones((N, A), np.int8)
    mask[::5, 1] = 0  # ragged legal sets
    mask[::7, 0] = 0
    pmask = (rng.uniform(size=N) > 0.2).astype(np.int32)
    seeds = torch.arange(S, dtype=torch.int32, device=DEV) * 7919
    cfg = dict(num_simulations=S, discount_factor=0.997, model=dict(support_scale=300, categorical_distribution=True))
    target, values = reanalyze_policy_targets(model, obs, torch.from_numpy(mask).to(DEV),
                                              torch.from_numpy(pmask).to(DEV), cfg, seeds=seeds)
    # the same search through the drop-in API
    legal = [list(np.nonzero(m)[0]) for m in mask]
    mcfg = MuZeroMCTSCtree.default_config()
    mcfg.update(cfg)
    mcfg.device = DEV
    mcts = MuZeroMCTSCtree(EasyDict(mcfg))
    with torch.no_grad():
        o = model.initial_inference(obs)
        roots = MuZeroMCTSCtree.roots(N, legal)
        tp = torch.full((N,), -1, dtype=torch.int32, device=DEV)
        roots.prepare_device(0.0, None, torch.zeros(N, device=DEV), o.policy_logits, tp)
        mcts.search(roots, model, o.latent_state, tp, seeds=seeds)
        dist = roots.get_distributions()
        vals = roots.get_values()
    tgt = target.cpu().numpy()
    for i in range(N):
        want = np.zeros(A, np.float32)
        if pmask[i]:
            d = np.asarray(dist[i], np.float64)
            for j, a in enumerate(legal[i]):
                want[a] = d[j] / d.sum()
        np.testing.assert_allclose(tgt[i], want, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(values.cpu().numpy(), np.asarray(vals, np.float32))


def test_roots_from_action_mask_equal_list_roots():
    """Roots.from_action_mask (legal lists built on the device) == Roots(n, host lists): the same
    device legal table and count, the same host list view, and the same prepared root priors"""
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    rng = np.random.default_rng(3)
    N, A = 257, 6
    mask = (rng.uniform(size=(N, A)) > 0.4).astype(np.int8)
    mask[5] = 0  # an empty row: every action legal (cnode.cpp:100-107), count 0 on both sides
    lists = [[i for i, x in enumerate(row) if x == 1] for row in mask]
    r1 = MuZeroMCTSCtree.roots(N, lists)
    r2 = MuZeroMCTSCtree.roots_from_mask(torch.from_numpy(mask).to(DEV))
    _, l1, c1 = r1.device_legal(A, DEV)
    _, l2, c2 = r2.device_legal(A, DEV)
    assert torch.equal(l1, l2) and torch.equal(c1, c2)
    assert r2.legal_actions_list == lists
    logits = torch.randn(N, A, device=DEV)
    z = torch.zeros(N, device=DEV)
    tp = torch.full((N,), -1, dtype=torch.int32, device=DEV)
    for r in (r1, r2):
        r.prepare_device(0.0, None, z, logits, tp)
    assert r1.get_distributions() == r2.get_distributions()
    s1 = r1.tree.dump_stats() if hasattr(r1.tree, "dump_stats") else None
    assert s1 is None or torch.equal(s1, r2.tree.dump_stats())
