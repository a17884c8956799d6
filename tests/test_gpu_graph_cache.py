"""GPU: captured-search caches stay correct when batch size, model or parameters change.

A search replayed as a HIP graph (cfg.use_hip_graph) reads the buffers and the folded network it
was captured over. These tests alternate what the captured graphs depend on — the batch size
(B = 8 -> 16 -> 8), the model (m1 -> m2 -> m1), the model's parameters (an in-place update between
replays) — and check every graph result against the eager loop on the same inputs and seeds
(visit counts and trajectories bit-exact, root values bit-exact: same kernels, same order).
Also: the AlphaZero graph cache keyed on a bound method replays instead of re-capturing, and the
collect step picks up a parameter update without re-capture.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from tests.test_gpu_conv import conv_model, run_search  # noqa: E402
from tests.test_gpu_search import CategoricalModel  # noqa: E402

DEV = torch.device("cuda", 0)


def _generic_search(mcts, model, B, S, A, seed):
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    rng = np.random.default_rng(seed)
    lat0 = rng.normal(size=(B, 32)).astype(np.float32)
    logits0 = rng.normal(size=(B, A)).astype(np.float32)
    noises = rng.dirichlet([0.3] * A, size=B).astype(np.float32)
    roots = MuZeroMCTSCtree.roots(B, [list(range(A))] * B)
    roots.prepare(0.25, [n.tolist() for n in noises], [0.0] * B, logits0.tolist(), [-1] * B)
    set_seed_source(SequentialSeeds(seed))
    try:
        mcts.search(roots, model, lat0, [-1] * B)
    finally:
        set_seed_source(None)
    out = (np.asarray(roots.get_distributions()), np.asarray(roots.get_values(), np.float32),
           roots.get_trajectories())
    roots.clear()
    return out


def _mcts(S, graph):
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    return MuZeroMCTSCtree(EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, use_hip_graph=graph,
                                         model=dict(support_scale=300, categorical_distribution=True))))


def test_graph_cache_alternating_batch_sizes_and_models_equal_eager():
    S, A = 12, 4
    m1, m2 = CategoricalModel(32, A, seed=1).to(DEV), CategoricalModel(32, A, seed=2).to(DEV)
    g, e = _mcts(S, True), _mcts(S, False)
    for i, (B, m) in enumerate([(8, m1), (16, m1), (8, m1), (8, m2), (16, m2), (8, m1), (16, m1)]):
        got = _generic_search(g, m, B, S, A, seed=10 + i)
        ref = _generic_search(e, m, B, S, A, seed=10 + i)
        assert np.array_equal(got[0], ref[0]), f"call {i} (B={B}): visit counts differ from eager"
        assert np.array_equal(got[1], ref[1]), f"call {i} (B={B}): root values differ from eager"
        assert got[2] == ref[2], f"call {i} (B={B}): trajectories differ from eager"
    assert len(g._graphs) <= g._graphs.cap


def test_graph_cache_is_bounded():
    S, A = 6, 4
    m = CategoricalModel(32, A, seed=3).to(DEV)
    g = _mcts(S, True)
    g._graphs.cap = 2
    for B in (4, 8, 12, 16, 4):
        _generic_search(g, m, B, S, A, seed=B)
    assert len(g._graphs) == 2


def test_graph_cache_conv_models_alternate_and_parameter_update():
    """Folded conv networks: m1 -> m2 -> m1 with the graph path equals eager; an in-place parameter
    update of m1 between replays is picked up (the captured graph reads the re-folded weights)."""
    B, S = 8, 10
    m1, m2 = conv_model("mz", seed=0), conv_model("mz", seed=5)
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    cfg = dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
               model=dict(support_scale=300, categorical_distribution=True))
    g = MuZeroMCTSCtree(EasyDict(dict(cfg, use_hip_graph=True)))
    e = MuZeroMCTSCtree(EasyDict(dict(cfg, use_hip_graph=False)))

    def both(m, seed):
        a = run_search("mz", B, S, seed, graph=True, record=False, model=m, mcts=g)
        b = run_search("mz", B, S, seed, graph=False, record=False, model=m, mcts=e)
        return a, b

    for i, m in enumerate([m1, m2, m1]):
        a, b = both(m, 20 + i)
        assert np.array_equal(a["dist"], b["dist"]) and np.array_equal(a["values"], b["values"]), f"model switch {i}"
    with torch.no_grad():
        for p in m1.prediction_network.parameters():
            p.mul_(1.5)
    a, b = both(m1, 30)
    assert np.array_equal(a["dist"], b["dist"]) and np.array_equal(a["values"], b["values"]), "after update"


def test_alphazero_graph_cache_keyed_on_bound_method():
    from lightzero_amd.alphazero import AlphaZeroMCTS
    from lightzero_amd.model_az import AlphaZeroModel
    torch.manual_seed(0)
    net = AlphaZeroModel().to(DEV).eval()
    mcts = AlphaZeroMCTS(num_simulations=8, device=DEV, graph=True)
    boards = np.zeros((4, 9), np.int32)
    for _ in range(3):
        mcts.get_next_actions(boards, [0] * 4, net.compute_policy_value)  # a new bound method each time
    assert len(mcts._buffers(4)["graphs"]) == 1


def test_collect_step_picks_up_parameter_update():
    """DeviceSearchStep replays one captured graph; after an in-place parameter update the replay
    must equal a freshly built step over the updated model (same seeds)."""
    from lightzero_amd.collect import DeviceSearchStep
    from lightzero_amd.model_mlp import cartpole_muzero_model
    B, S = 16, 10
    torch.manual_seed(0)
    m = cartpole_muzero_model(random_heads=True).to(DEV).eval()
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32)).to(DEV)
    noises = torch.from_numpy(rng.dirichlet([0.3, 0.3], size=B).astype(np.float32)).to(DEV)

    def fresh():
        st = DeviceSearchStep(m, B, S, [[0, 1]] * B, (4,), DEV, seed=3)
        st.set_inputs(obs=obs, noises=noises)
        return st

    st = fresh()
    st.step()
    st.reset_seed_counter()
    with torch.no_grad():
        for p in m.dynamics_network.parameters():
            p.mul_(0.5)
        for p in m.representation_network.parameters():
            p.add_(0.01)
    out = st.step()
    d1, v1 = out["distributions"].clone(), out["values"].clone()
    ref = fresh()
    ref.build_graph()
    ref.reset_seed_counter()
    out2 = ref.step()
    assert torch.equal(d1, out2["distributions"]) and torch.equal(v1, out2["values"])
