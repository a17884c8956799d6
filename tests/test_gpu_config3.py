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
