"""GPU: the device collect loop (lzm_cartpole_* kernels, lightzero_amd.collector.DeviceCollector).

Env parity is unpinned (gymnasium is absent): the device CartPole is checked against the numpy
restatement of the same published equations (oracle/cartpole.py) to float64 round-off; action
sampling and Dirichlet noise (Philox streams, not numpy's) are checked statistically.
"""
import numpy as np
import pytest
import torch

from oracle import cartpole

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _raw_step(n, visits, state, steps, obs, counter, temperature=1.0, deterministic=1, T=200, E=4, seed=5):
    from lightzero_amd._lib import call, ptr, stream_ptr
    A = visits.shape[1]
    rec = dict(obs=torch.zeros((n, E, T + 1, 4), device=DEV), action=torch.zeros((n, E, T), dtype=torch.int32,
                                                                                  device=DEV),
               reward=torch.zeros((n, E, T), device=DEV), child=torch.zeros((n, E, T, A), dtype=torch.int32, device=DEV),
               value=torch.zeros((n, E, T), device=DEV), ep_len=torch.zeros((n, E), dtype=torch.int32, device=DEV),
               ep_count=torch.zeros(n, dtype=torch.int32, device=DEV))
    noises = torch.zeros((n, A), device=DEV)
    value = torch.zeros(n, device=DEV)
    call("lzm_cartpole_collect_step", n, A, T, E, ptr(visits), ptr(value), None, ptr(state), ptr(steps), ptr(obs),
         ptr(noises), 0.3, float(temperature), int(deterministic), ptr(rec["obs"]), ptr(rec["action"]),
         ptr(rec["reward"]), ptr(rec["child"]), ptr(rec["value"]), None, ptr(rec["ep_len"]), ptr(rec["ep_count"]), None,
         T, seed, ptr(counter), stream_ptr())
    return rec, noises


def test_cartpole_physics_matches_numpy_restatement():
    n = 64
    rng = np.random.default_rng(0)
    s0 = rng.uniform(-0.05, 0.05, size=(n, 4))
    state = torch.from_numpy(s0.copy()).to(DEV)
    steps = torch.zeros(n, dtype=torch.int32, device=DEV)
    obs = state.float().clone()
    counter = torch.zeros(1, dtype=torch.int64, device=DEV)
    ref = s0.copy()
    alive = np.ones(n, bool)
    for k in range(40):
        acts = rng.integers(0, 2, size=n)
        visits = torch.from_numpy(np.stack([1 - acts, acts], 1).astype(np.int32)).to(DEV)  # argmax = acts
        rec, _ = _raw_step(n, visits, state, steps, obs, counter, deterministic=1)
        counter += 1
        got = state.cpu().numpy()
        for i in range(n):
            if not alive[i]:
                continue
            ref[i], term = cartpole.step(ref[i], int(acts[i]))
            if term:
                alive[i] = False  # the device env reset this one
                assert int(rec["ep_len"][i, 0]) == k + 1
                continue
            np.testing.assert_allclose(got[i], ref[i], rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(obs[i].cpu().numpy(), ref[i].astype(np.float32), rtol=1e-6, atol=1e-9)
    assert (~alive).any(), "some episodes should terminate within 40 random steps"


def test_select_action_sampling_frequencies():
    n, S = 20000, 50
    a0 = 15
    visits = torch.tensor([[a0, S - a0]] * n, dtype=torch.int32, device=DEV)
    state = torch.zeros((n, 4), dtype=torch.float64, device=DEV)
    steps = torch.zeros(n, dtype=torch.int32, device=DEV)
    obs = torch.zeros((n, 4), device=DEV)
    counter = torch.zeros(1, dtype=torch.int64, device=DEV)
    for T, p0 in [(1.0, a0 / S), (0.5, a0 ** 2 / (a0 ** 2 + (S - a0) ** 2))]:
        rec, noises = _raw_step(n, visits, state, steps, obs, counter, temperature=T, deterministic=0)
        frac = float((rec["action"][:, 0, 0] == 0).float().mean())
        sd = (p0 * (1 - p0) / n) ** 0.5
        assert abs(frac - p0) < 5 * sd, (T, frac, p0)
        nz = noises.cpu().numpy()
        assert np.allclose(nz.sum(1), 1.0, atol=1e-6) and (nz > 0).all()
        assert abs(nz[:, 0].mean() - 0.5) < 0.02  # Dirichlet(0.3, 0.3): mean 1/2
        counter += 1
        steps.zero_()


@pytest.mark.parametrize("graph", [True, False])
def test_device_collector_episodes(graph):
    from lightzero_amd.collector import DeviceCollector
    from tests.test_gpu_collect import _model
    n, S = 32, 16
    col = DeviceCollector(_model(), n, S, device=DEV, seed=3, graph=graph, poll_every=4)
    eps, stats = col.collect(n_episode=n)
    assert len(eps) >= n and stats["envstep"] > 0
    for e in eps:
        L = len(e["action_segment"])
        assert 1 <= L <= 200
        assert e["obs_segment"].shape == (L + 1, 4)
        assert np.all(np.abs(e["obs_segment"][0]) <= 0.05 + 1e-7)
        assert set(np.unique(e["action_segment"])) <= {0, 1}
        np.testing.assert_allclose(e["child_visit_segment"].sum(1), 1.0, atol=1e-6)
        np.testing.assert_allclose(e["child_visit_segment"] * S, np.round(e["child_visit_segment"] * S), atol=1e-4)
        assert (e["reward_segment"] == 1.0).all()
        last = e["obs_segment"][L]
        if L < 200:  # terminated: the final state is outside the thresholds
            assert abs(last[0]) > cartpole.X_THRESHOLD or abs(last[2]) > cartpole.THETA_THRESHOLD - 1e-6
        # replay the recorded actions through the numpy restatement from the recorded first obs
        s = e["obs_segment"][0].astype(np.float64)
        for t in range(min(L, 10)):
            s, _ = cartpole.step(s, int(e["action_segment"][t]))
            np.testing.assert_allclose(s.astype(np.float32), e["obs_segment"][t + 1], rtol=1e-4, atol=1e-5)


def test_device_collector_graph_equals_eager():
    from lightzero_amd.collector import DeviceCollector
    from tests.test_gpu_collect import _model
    n, S = 16, 12
    model = _model()
    out = []
    for graph in (True, False):
        col = DeviceCollector(model, n, S, device=DEV, seed=9, graph=graph, poll_every=2)
        for _ in range(20):
            col.step()
        torch.cuda.synchronize()
        out.append((col.rec_action.cpu().numpy(), col.rec_visits.cpu().numpy(), col.env.state.cpu().numpy()))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
