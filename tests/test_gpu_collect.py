"""GPU: the graph-captured collect step (lightzero_amd.collect.DeviceSearchStep).

Each replay must equal, bit for bit, the Python-driven sequence it captures —
initial_inference -> Roots.prepare_device -> MuZeroMCTSCtree.search with the host
SequentialSeeds source (usec_k = (1000003*seed + k) mod 1e6 over consecutive traverses) ->
distributions / values — for several consecutive steps (the device seed counter advances).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _model(seed=0):
    from lightzero_amd.model_mlp import cartpole_muzero_model
    torch.manual_seed(seed)
    m = cartpole_muzero_model(random_heads=True)
    g = torch.Generator().manual_seed(seed + 1)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            with torch.no_grad():
                mod.running_mean.copy_(torch.randn(mod.running_mean.shape, generator=g) * 0.1)
                mod.running_var.copy_(torch.rand(mod.running_var.shape, generator=g) * 0.5 + 0.75)
    return m.to(DEV).eval()


def _reference_steps(model, obs_list, noises_list, B, S, seed, legal):
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.utils import EasyDict
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV,
                        model=dict(support_scale=300, categorical_distribution=True)))
    mcts = MuZeroMCTSCtree(cfg)
    set_seed_source(SequentialSeeds(seed))
    outs = []
    try:
        for obs, nz in zip(obs_list, noises_list):
            with torch.no_grad():
                o = model.initial_inference(obs)
                roots = MuZeroMCTSCtree.roots(B, legal)
                tp = torch.full((B,), -1, dtype=torch.int32, device=DEV)
                roots.prepare_device(0.25, nz, torch.zeros(B, device=DEV), o.policy_logits, tp)
                mcts.search(roots, model, o.latent_state, tp)
                outs.append((roots.tree.distributions().cpu().numpy(), roots.tree.values().cpu().numpy()))
                roots.clear()
    finally:
        set_seed_source(None)
    return outs


# the collect-step glue (seeds from the step counter, fresh min-max, root outputs, counter) runs
# inside the network-resident kernel, and around the weight-streaming kernel (LZM_FUSED_RES=0)
@pytest.mark.parametrize("env", ["", "LZM_FUSED_RES=0"])
@pytest.mark.parametrize("graph", [False, True])
def test_device_search_step_matches_python_search(graph, env, monkeypatch):
    if env:
        monkeypatch.setenv(*env.split("="))
    from lightzero_amd.collect import DeviceSearchStep
    B, S, seed = 64, 30, 7
    legal = [[0, 1]] * B
    model = _model()
    rng = np.random.default_rng(0)
    obs_list = [torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32)).to(DEV) for _ in range(3)]
    nz_list = [torch.from_numpy(rng.dirichlet([0.3, 0.3], size=B).astype(np.float32)).to(DEV) for _ in range(3)]
    ref = _reference_steps(model, obs_list, nz_list, B, S, seed, legal)
    step = DeviceSearchStep(model, B, S, legal, (4,), DEV, seed=seed, graph=graph)
    for k, (obs, nz) in enumerate(zip(obs_list, nz_list)):
        step.set_inputs(obs=obs, noises=nz)
        out = step.step()
        d, v = out["distributions"].cpu().numpy(), out["values"].cpu().numpy()
        assert np.array_equal(d, ref[k][0]), f"step {k}: visit counts differ"
        assert np.array_equal(v, ref[k][1]), f"step {k}: root values differ"
        assert (d.sum(axis=1) == S).all()
        assert int(step.step_counter.item()) == k + 1
