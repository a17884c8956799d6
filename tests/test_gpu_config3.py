"""GPU: config 3's collect-time step (BASELINE.json config 3, Pong EfficientZero; reference
lzero/policy/efficientzero.py:538-656 _forward_collect, mcts_ctree.py:696-827): the BN-folded conv
initial inference of the EfficientZeroModel, root preparation with the value-prefix roots, the one-launch
EZ search (lzm_search_conv_ez) handed the initial inference's reward_hidden_state, and the root outputs —
as lightzero_amd.collect.DeviceSearchStep, eagerly and captured as one HIP graph.

Parity: the step equals EfficientZeroMCTSCtree.search called with the same seeds and roots (bit for bit;
that search is oracle-exact, tests/test_gpu_conv.py), and the captured graph equals the eager step.
"""
import numpy as np
import pytest
import torch

import bench

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _ez_model(seed=0):
    from lightzero_amd.model_conv import atari_efficientzero_model
    torch.manual_seed(seed)
    m = atari_efficientzero_model(last_linear_layer_init_zero=False)
    bench._random_bn(m, seed + 1)
    return m.to(DEV).eval()


def _inputs(B, seed):
    rng = np.random.default_rng(seed)
    obs = torch.from_numpy(bench.synthetic_obs("breakout", B, rng)).to(DEV)
    noises = torch.from_numpy(rng.dirichlet([0.3] * 6, size=B).astype(np.float32)).to(DEV)
    return obs, noises


@pytest.mark.parametrize("B,S", [(64, 20), (256, 50)])
def test_ez_collect_step_equals_plain_search(B, S):
    from lightzero_amd.collect import DeviceSearchStep
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    seed = 6
    model = _ez_model(3)
    obs, noises = _inputs(B, seed)
    step = DeviceSearchStep(model, B, S, [list(range(6))] * B, (4, 64, 64), DEV, seed=seed, graph=False,
                            support_scale=50)
    assert step.ez and step.mcts_cls is EfficientZeroMCTSCtree
    step.set_inputs(obs=obs, noises=noises)
    outs = []
    for _ in range(2):
        o = step.step()
        outs.append((o["distributions"].clone(), o["values"].clone()))
    assert step.mcts.last_path == "fused"
    assert all(int(d.sum()) == B * S for d, _ in outs)
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                        model=dict(support_scale=50, categorical_distribution=True)))
    mcts = EfficientZeroMCTSCtree(cfg)
    base = (1000003 * seed) % 1000000
    to_play = torch.full((B,), -1, dtype=torch.int32, device=DEV)
    with torch.no_grad():
        for n, (dist, vals) in enumerate(outs):
            out = step.initial.initial_inference(obs)  # (the step's BN-folded initial inference)
            roots = EfficientZeroMCTSCtree.roots(B, [list(range(6))] * B)
            roots.prepare_device(0.25, noises, torch.zeros(B, device=DEV), out.policy_logits, to_play)
            seeds = torch.tensor([(base + n * S + k) % 1000000 for k in range(S)], dtype=torch.int32, device=DEV)
            mcts.search(roots, model, out.latent_state, out.reward_hidden_state, to_play, seeds=seeds)
            assert mcts.last_path == "fused"
            assert torch.equal(roots.tree.distributions(), dist)
            assert torch.equal(roots.tree.values(), vals)
            roots.clear()


def test_ez_collect_step_graph_equals_eager():
    from lightzero_amd.collect import DeviceSearchStep
    B, S = 48, 16
    model = _ez_model(4)
    obs, noises = _inputs(B, 9)
    res = []
    for graph in (False, True):
        step = DeviceSearchStep(model, B, S, [list(range(6))] * B, (4, 64, 64), DEV, seed=2, graph=graph,
                                support_scale=50)
        step.set_inputs(obs=obs, noises=noises)
        got = []
        for _ in range(3):  # fresh seeds each replay (the device step counter)
            o = step.step()
            got.append((o["distributions"].clone(), o["values"].clone()))
        torch.cuda.synchronize()
        step.roots.tree.check_errors()
        res.append(got)
    for (d0, v0), (d1, v1) in zip(*res):
        assert torch.equal(d0, d1) and torch.equal(v0, v1)


# ---- the device collect step of config 3 (DeviceCollector(env="pong") on the EfficientZero model) ------------
def _pong_collector(n=32, S=8, T=120, E=8, seed=3, graph=True, model=None):
    from lightzero_amd.collector import DeviceCollector
    return DeviceCollector(model or _ez_model(3), n, S, device=DEV, seed=seed, graph=graph, poll_every=4,
                           episode_slots=E, max_episode_steps=T, env="pong")


def test_pong_collect_searches_equal_plain_search():
    """the device collector's EfficientZero collect step (graph-captured: initial inference, the one-launch EZ
    search in collect-step mode, the Pong stand-in's env step) — each step's search, re-run through
    EfficientZeroMCTSCtree.search on the same observation stack, noises and device seeds, gives the same visit
    counts and root values bit for bit (the env step between searches included)"""
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    B, S, seed = 48, 12, 5
    col = _pong_collector(n=B, S=S, seed=seed)
    assert col.search.ez and col.A == 6
    recs = []
    for _ in range(6):
        obs, noises = col.search.obs.clone(), col.search.noises.clone()
        col.step()
        o = col.search.out
        recs.append((obs, noises, o["distributions"].clone(), o["values"].clone()))
    torch.cuda.synchronize()
    assert col.search.mcts.last_path == "fused"
    col.search.roots.tree.check_errors()
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                        model=dict(support_scale=50, categorical_distribution=True)))
    mcts = EfficientZeroMCTSCtree(cfg)
    base = (1000003 * seed) % 1000000
    to_play = torch.full((B,), -1, dtype=torch.int32, device=DEV)
    with torch.no_grad():
        for n, (obs, noises, dist, vals) in enumerate(recs):
            out = col.search.initial.initial_inference(obs)
            roots = EfficientZeroMCTSCtree.roots(B, [list(range(6))] * B)
            roots.prepare_device(0.25, noises, torch.zeros(B, device=DEV), out.policy_logits, to_play)
            seeds = torch.tensor([(base + n * S + k) % 1000000 for k in range(S)], dtype=torch.int32, device=DEV)
            mcts.search(roots, col.search.model, out.latent_state, out.reward_hidden_state, to_play, seeds=seeds)
            assert mcts.last_path == "fused"
            assert torch.equal(roots.tree.distributions(), dist), n
            assert torch.equal(roots.tree.values(), vals), n
            roots.clear()


def test_pong_episodes_replay_through_the_restated_game():
    """the Pong stand-in's recorded episodes (u8 frames, actions, clipped rewards, the point difference as the
    return) re-derive through its numpy restatement (oracle/pong_synth.py); visit counts sum to S"""
    from oracle import pong_synth
    col = _pong_collector()
    blocks, stats = col.collect_blocks(n_episode=32, to_host=True)
    (b,) = blocks
    assert b.frames.dtype == np.uint8 and b.frames.shape[1:] == (1, 64, 64)
    assert stats["episodes"] == b.num_episodes >= 32
    for env_id, L, r0 in b.index:
        sc = b.scalars[r0:r0 + L + 1]
        fr = b.frames[r0:r0 + L + 1]
        actions, rewards = np.rint(sc[:L, 0]).astype(np.int64), sc[:L, 1]
        assert 1 <= L <= col.T and set(np.unique(actions)) <= set(range(6))
        assert set(np.unique(rewards)) <= {-1.0, 0.0, 1.0}
        assert (sc[:L, 2:8].sum(axis=1) == col.S).all()
        assert sc[L, 0] == 0 and (sc[L, 2:] == 0).all() and sc[L, 1] == rewards.sum()
        msg = pong_synth.replay_episode(fr, actions, rewards, col.T, episode_return=sc[L, 1])
        assert msg is None, f"env {env_id} episode of {L} steps: {msg}"


def test_pong_collect_graph_equals_eager():
    """the captured collect step (search + env step in one HIP graph) equals the eager one: actions, frames,
    visit counts"""
    out = []
    for graph in (False, True):
        col = _pong_collector(n=16, S=8, T=60, seed=9, graph=graph)
        for _ in range(12):
            col.step()
        torch.cuda.synchronize()
        out.append((col.rec_action.cpu().numpy(), col.rec_visits.cpu().numpy(), col.env.state.cpu().numpy(),
                    col.rec_frames.cpu().numpy()))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
