"""GPU: the MuZeroCollector drop-in (lightzero_amd.worker) against the host restatement of the
reference's collect loop (oracle/collector_ref.py).

Host-parity mode — MuZeroCollector's host loop over MuZeroCollectPolicy (GPU search, numpy noise
and action draws): on the same numpy seed and traverse seeds, the restatement — the reference's
loop and _forward_collect with the ORACLE tree replaying the network outputs the GPU search
recorded — issues the same tree requests, draws the same noises, picks the same actions and
returns identical segments (observations, actions, rewards, visit distributions, root values,
masks, players), priorities and done flags. At the config-1 shape (8 envs x 25 sims) and the
headline shape (256 x 50), with segment rollover exercised (game_segment_length 7 and 50).

Device path — DeviceCartPoleEnvManager (the graph-captured device collector, Philox streams): the
episodes the device played, replayed through the restatement, give the segments, priorities,
flags and pool order the collector returned (n_episode == env_num and > env_num).
"""
import numpy as np
import pytest
import torch

from oracle.collector_ref import EpisodeEnv, EpisodeForward, ReplayForward, ref_collect

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


def _eq(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.dtype == b.dtype, (what, a.dtype, b.dtype)
    assert a.shape == b.shape and np.array_equal(a, b), what


def _compare(segs, meta, ref_segs, ref_meta):
    assert len(segs) == len(ref_segs) and len(meta) == len(ref_meta)
    for g, r in zip(segs, ref_segs):
        for f in ("obs_segment", "action_segment", "reward_segment", "child_visit_segment", "root_value_segment",
                  "action_mask_segment", "to_play_segment"):
            _eq(getattr(g, f), r[f], f)
    for m, rm in zip(meta, ref_meta):
        assert m['done'] == rm['done'] and m['unroll_plus_td_steps'] == rm['unroll_plus_td_steps']
        if rm['priorities'] is None:
            assert m['priorities'] is None
        else:
            _eq(m['priorities'], rm['priorities'], 'priorities')


@pytest.mark.parametrize("n,S,gsl", [(8, 25, 50), (8, 25, 7), (256, 50, 50)])
def test_parity_mode_matches_host_restatement(n, S, gsl):
    from lightzero_amd.envs import SyncEnvManager
    from lightzero_amd.policy import MuZeroCollectPolicy, policy_config
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.worker import MuZeroCollector
    cfg = policy_config(num_simulations=S, game_segment_length=gsl, device=DEV, use_priority=True, n_episode=n)
    policy = MuZeroCollectPolicy(cfg, _model(1))
    policy.record = True
    set_seed_source(SequentialSeeds(11))
    np.random.seed(123)
    try:
        col = MuZeroCollector(env=SyncEnvManager.cartpole(n, seed=5), policy=policy, policy_config=cfg)
        segs, meta = col.collect(n_episode=n, policy_kwargs=dict(temperature=1.0, epsilon=0.0))
    finally:
        set_seed_source(None)
    np.random.seed(123)
    fwd = ReplayForward(cfg, policy.records)
    ref_segs, ref_meta, st = ref_collect(cfg, SyncEnvManager.cartpole(n, seed=5), fwd, n)
    assert fwd.mismatch == [], fwd.mismatch[:5]
    assert fwd.k == len(policy.records)
    _compare(segs, meta, ref_segs, ref_meta)
    assert col.envstep == st["steps"] and len(segs) >= n
    # the visit counts behind the segments sum to the simulations
    for r in policy.records:
        assert all(sum(d) == S for d in r["dist"])


def _played(sched):
    return [[dict(obs=e["obs_segment"], action=e["action_segment"], reward=e["reward_segment"], visits=e["visits"],
                  value=e["root_value_segment"], pred=e.get("pred_value_segment")) for e in eps] for eps in sched.played]


@pytest.mark.parametrize("n,n_ep,gsl,prio", [(16, 16, 10, True), (32, 48, 50, False), (64, 64, 50, True)])
def test_device_path_segments_match_restatement(n, n_ep, gsl, prio):
    from lightzero_amd.envs import DeviceCartPoleEnvManager
    from lightzero_amd.policy import MuZeroCollectPolicy, policy_config
    from lightzero_amd.worker import MuZeroCollector
    cfg = policy_config(num_simulations=12, game_segment_length=gsl, device=DEV, use_priority=prio, n_episode=n)
    col = MuZeroCollector(env=DeviceCartPoleEnvManager(n, seed=3), policy=MuZeroCollectPolicy(cfg, _model(2)),
                          policy_config=cfg)
    seen = []
    for temperature in (1.0, 0.5):
        segs, meta = col.collect(n_episode=n_ep, policy_kwargs=dict(temperature=temperature, epsilon=0.0))
        sched = col.last_schedule
        eps = _played(sched)
        assert sum(len(e) for e in eps) == n_ep and all(len(e) >= 1 for e in eps)
        env = EpisodeEnv(eps)
        ref_segs, ref_meta, st = ref_collect(cfg, env, EpisodeForward(env), n_ep)
        _compare(segs, meta, ref_segs, ref_meta)
        for e in sum(eps, []):
            assert (e["visits"].sum(axis=1) == 12).all() and (e["reward"] == 1.0).all()
            assert np.all(np.abs(e["obs"][0]) <= 0.05 + 1e-7)
        # the logged episode return is CartPole's reward sum (eval_episode_return), one per counted episode
        info = col._episode_info[-n_ep:]
        assert [d['reward'] for d in info] == [float(d['step']) for d in info]
        seen.append(segs[0].obs_segment.copy())
    assert not np.array_equal(seen[0], seen[1])  # the second collect plays fresh episodes


def test_device_path_breakout_segments_match_restatement():
    """config 5's device path through the MuZeroCollector drop-in: the Breakout stand-in env (u8 frames,
    frame_stack_num 4), episodes cut into segments whose observation windows stack 4 frames — identical
    to the restatement of the reference's loop fed the same episodes"""
    import bench
    from lightzero_amd.envs import DeviceBreakoutEnvManager
    from lightzero_amd.policy import MuZeroCollectPolicy, policy_config
    from lightzero_amd.worker import MuZeroCollector
    n, n_ep = 16, 24
    cfg = policy_config(num_simulations=8, game_segment_length=12, device=DEV, use_priority=True, n_episode=n,
                        model=dict(frame_stack_num=4, action_space_size=4, observation_shape=(4, 64, 64),
                                   image_channel=1, model_type='conv'))
    model = bench.build_conv_model(DEV, seed=3)
    col = MuZeroCollector(env=DeviceBreakoutEnvManager(n, seed=7, max_episode_steps=150),
                          policy=MuZeroCollectPolicy(cfg, model), policy_config=cfg)
    segs, meta = col.collect(n_episode=n_ep, policy_kwargs=dict(temperature=1.0, epsilon=0.0))
    eps = _played(col.last_schedule)
    assert sum(len(e) for e in eps) == n_ep
    env = EpisodeEnv(eps)
    ref_segs, ref_meta, _ = ref_collect(cfg, env, EpisodeForward(env), n_ep)
    _compare(segs, meta, ref_segs, ref_meta)
    for g in segs:
        assert g.obs_segment.shape[1:] == (1, 64, 64) and g.obs_segment.dtype == np.float32
        assert len(g.obs_segment) >= 4 + len(g.action_segment)
    for e in sum(eps, []):
        assert (e["visits"].sum(axis=1) == 8).all() and set(np.unique(e["reward"])) <= {0.0, 1.0}
    # the logged reward is each counted episode's UNCLIPPED score (eval_episode_return), as replayed
    # through the restated game; the clipped rewards only count the scoring steps
    from oracle import breakout_synth
    counted = [e for r in col.last_schedule.played for e in r]
    info = col._episode_info[-n_ep:]
    assert sorted(d['reward'] for d in info) == sorted(float(e["episode_return"]) for e in counted)
    for e in counted:
        fr = np.rint(e["obs_segment"] * 255).astype(np.uint8)
        assert e["episode_return"] >= e["reward_segment"].sum()
        assert breakout_synth.replay_episode(fr, e["action_segment"], e["reward_segment"], 150,
                                             episode_return=e["episode_return"]) is None


def test_device_path_pong_efficientzero_segments_match_restatement():
    """config 3's device path through the MuZeroCollector drop-in: an EfficientZeroCollectPolicy on the Pong
    stand-in (DevicePongEnvManager) takes the device collector (the one-launch EfficientZero search with the
    reward LSTM in the captured step, lstm_horizon_len from the policy config), and its episodes cut into
    segments identical to the restatement of the reference's loop fed the same episodes; the logged return is
    each counted episode's point difference"""
    import bench
    from lightzero_amd.envs import DevicePongEnvManager
    from lightzero_amd.policy import EfficientZeroCollectPolicy, policy_config
    from lightzero_amd.worker import MuZeroCollector
    from oracle import pong_synth
    n, n_ep = 16, 20
    cfg = policy_config(num_simulations=8, game_segment_length=12, device=DEV, use_priority=True, n_episode=n,
                        lstm_horizon_len=5,
                        model=dict(frame_stack_num=4, action_space_size=6, observation_shape=(4, 64, 64),
                                   image_channel=1, model_type='conv', support_scale=50))
    model = bench.build_ez_model(DEV, seed=3)
    col = MuZeroCollector(env=DevicePongEnvManager(n, seed=7, max_episode_steps=90),
                          policy=EfficientZeroCollectPolicy(cfg, model), policy_config=cfg)
    segs, meta = col.collect(n_episode=n_ep, policy_kwargs=dict(temperature=1.0, epsilon=0.0))
    assert col._device is not None and col._device.search.ez, "the EZ policy did not take the device path"
    assert col._device.search.mcts.last_path == "fused"
    eps = _played(col.last_schedule)
    assert sum(len(e) for e in eps) == n_ep
    env = EpisodeEnv(eps)
    ref_segs, ref_meta, _ = ref_collect(cfg, env, EpisodeForward(env), n_ep)
    _compare(segs, meta, ref_segs, ref_meta)
    for e in sum(eps, []):
        assert (e["visits"].sum(axis=1) == 8).all() and set(np.unique(e["reward"])) <= {-1.0, 0.0, 1.0}
    counted = [e for r in col.last_schedule.played for e in r]
    info = col._episode_info[-n_ep:]
    assert sorted(d['reward'] for d in info) == sorted(float(e["episode_return"]) for e in counted)
    for e in counted:
        fr = np.rint(e["obs_segment"] * 255).astype(np.uint8)
        assert e["episode_return"] == e["reward_segment"].sum()
        assert pong_synth.replay_episode(fr, e["action_segment"], e["reward_segment"], 90,
                                         episode_return=e["episode_return"]) is None
