"""GPU: the network-in-the-loop divergence at the headline config (BASELINE.json config 2: 256 envs x
50 sims, glibc parity mode) — VERDICT r03's parity gap.

The tree is bit-exact given the network outputs (every other search test), but the fused kernel's
network (BN folded, its own summation order) and the PyTorch module round differently (rtol 1e-4 on
the outputs), so two searches of the same weights, roots and seeds can part ways. This test runs both —
the one-launch fused search and the generic path with the torch MuZeroModelMLP in the loop — and:
  - replays each through the oracle with its own recorded network outputs (each reproduces exactly);
  - reports the fraction of roots whose visit counts differ;
  - attributes every root's FIRST divergent walk (tests/divergence.py) to a pUCT near-tie moved by
    rounding, or to a tie broken at a shifted position of the shared glibc rand() stream after an
    earlier root diverged — asserting nothing else occurs.
The numbers go to $LZM_REPORT_DIR/divergence_config2_*.json (profiles/ keeps the round's copy).
"""
import numpy as np
import pytest
import torch

import bench
from tests.divergence import attribute, report

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _search(model, fused, obs, noises, seed, B, S):
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.utils import EasyDict
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, use_hip_graph=False, fused_search=fused,
                        model=dict(support_scale=300, categorical_distribution=True)))
    mcts = MuZeroMCTSCtree(cfg)
    mcts.record = True
    with torch.no_grad():
        out = model.initial_inference(obs)
    logits0 = out.policy_logits.float().cpu().numpy()
    roots = MuZeroMCTSCtree.roots(B, [[0, 1]] * B)
    roots.prepare(0.25, noises.tolist(), [0.0] * B, logits0.tolist(), [-1] * B)
    set_seed_source(SequentialSeeds(seed))
    try:
        mcts.search(roots, model, out.latent_state, [-1] * B)
    finally:
        set_seed_source(None)
    res = dict(rec=mcts.last_record.numpy(), dist=np.array(roots.get_distributions()),
               values=np.array(roots.get_values(), np.float32), noises=noises, logits0=logits0,
               path=mcts.last_path)
    roots.clear()
    return res


@pytest.mark.parametrize("heads", ["random", "zero"])
def test_fused_vs_torch_network_search_divergence_config2(heads):
    B, S = 256, 50
    model = bench.build_model(DEV, heads == "zero", seed=0)
    rng = np.random.default_rng(21)
    obs = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32)).to(DEV)
    noises = rng.dirichlet([0.3, 0.3], size=B).astype(np.float32)
    fused = _search(model, True, obs, noises, 5, B, S)
    torch_net = _search(model, False, obs, noises, 5, B, S)
    assert fused["path"] == "fused-mlp" and torch_net["path"] == "generic"
    rep = attribute(fused, torch_net, B, S, 2, tau=1e-4)
    report(f"config2_{heads}_heads", rep)
    kinds = rep["first_divergence_kinds"]
    assert kinds.get("unexplained", 0) == 0, rep["first_divergences"][:5]
    # a root whose walk diverges first, with no earlier root diverged, can only do so at a near-tie
    assert kinds.get("tie_draw", 0) == 0, [r for r in rep["first_divergences"] if r["kind"] == "tie_draw"][:3]
    assert (fused["dist"].sum(axis=1) == S).all() and (torch_net["dist"].sum(axis=1) == S).all()
    # measured (profiles/r04/divergence_config2_*.json): no root's visit counts differ; a few walks part
    # at near-ties (gaps ~1e-5) and the shared rand() stream then shifts for later roots, but the counts
    # re-converge. Bound the rate well above that, far below a real divergence.
    assert rep["rate"] <= 0.02, rep["rate"]
