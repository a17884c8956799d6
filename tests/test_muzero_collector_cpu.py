"""CPU: MuZeroCollector's segment assembly against the host restatement of the reference's collect
loop (oracle/collector_ref.py: muzero_collector.py:305-705, game_segment.py:129-294).

Both the collector's host loop and its device path's vectorised cutter (EpisodeSchedule +
episode_segments) are driven by the same recorded episodes — an env manager replaying them and a
policy replaying their search outputs — and must return identical segments (every field, dtype
included), priorities, done flags and pool order. Covered: segment rollover and pad_over at several
game_segment_length / num_unroll_steps / td_steps, frame stacking, episodes shorter than, equal
to and multiples of the segment length, n_episode == env_num and > env_num (envs handed new
episodes by remain_episode), priorities on/off, ignore_done.
"""
import numpy as np
import pytest
import torch

from oracle.collector_ref import EpisodeEnv, EpisodeForward, ref_collect

from lightzero_amd.envs import Discrete
from lightzero_amd.policy import policy_config
from lightzero_amd.worker import MuZeroCollector
from lightzero_amd.worker.segments import EpisodeSchedule, episode_segments

A = 2


def _episode(rng, L, pred=True):
    return dict(obs=rng.normal(size=(L + 1, 4)).astype(np.float32), action=rng.integers(0, A, size=L),
                reward=np.ones(L, np.float32), visits=rng.integers(0, 12, size=(L, A)).astype(np.int64),
                value=rng.normal(size=L).astype(np.float32),
                pred=rng.normal(size=L).astype(np.float32) if pred else None)


def _lengths(rng, gsl):
    pool = [1, 2, gsl - 1, gsl, gsl + 1, 2 * gsl, 2 * gsl + 3, 3 * gsl]
    return [int(rng.choice(pool)) if rng.random() < 0.6 else int(rng.integers(1, 3 * gsl + 2)) for _ in range(12)]


class _ReplayPolicy:
    """collect-mode surface over EpisodeForward (the collector calls forward / reset / get_attribute)"""

    def __init__(self, cfg, env):
        self.cfg, self.fwd = cfg, EpisodeForward(env)

    def forward(self, data, action_mask, temperature, to_play, epsilon, ready_env_id=None):
        return self.fwd(data, action_mask, temperature, to_play, epsilon, list(ready_env_id))

    def reset(self, *a, **k):
        return None

    def get_attribute(self, name):
        return self.cfg


class _Env(EpisodeEnv):
    action_space = Discrete(A)

    def launch(self):
        pass

    def reset(self, *a):
        pass

    def close(self):
        pass


def _eq(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.dtype == b.dtype, (what, a.dtype, b.dtype)
    assert a.shape == b.shape and np.array_equal(a, b), what


def _compare(segs, meta, ref_segs, ref_meta):
    assert len(segs) == len(ref_segs)
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


CASES = [  # (env_num, n_episode, gsl, U, TD, fs, use_priority, ignore_done)
    (3, 3, 5, 5, 5, 1, False, False),
    (4, 4, 7, 3, 2, 1, True, False),
    (4, 9, 5, 5, 5, 1, True, False),
    (5, 13, 4, 2, 3, 4, False, False),
    (3, 7, 6, 5, 3, 1, True, True),
    (6, 6, 50, 5, 5, 1, False, False),
]


def _cfg(gsl, U, TD, fs, prio, ign):
    return policy_config(game_segment_length=gsl, num_unroll_steps=U, td_steps=TD, use_priority=prio, ignore_done=ign,
                         device='cpu', model=dict(frame_stack_num=fs, observation_shape=4 * fs))


@pytest.mark.parametrize("case", CASES)
def test_host_loop_matches_restatement(case):
    n, n_ep, gsl, U, TD, fs, prio, ign = case
    rng = np.random.default_rng(sum(case[:5]))
    eps = [[_episode(rng, L) for L in _lengths(rng, gsl)] for _ in range(n)]
    cfg = _cfg(gsl, U, TD, fs, prio, ign)
    env_r = _Env(eps)
    ref_segs, ref_meta, st = ref_collect(cfg, env_r, EpisodeForward(env_r), n_ep)
    env = _Env(eps)
    col = MuZeroCollector(env=env, policy=_ReplayPolicy(cfg, env), policy_config=cfg)
    segs, meta = col.collect(n_episode=n_ep, policy_kwargs=dict(temperature=1.0, epsilon=0.0))
    _compare(segs, meta, ref_segs, ref_meta)
    assert env.k == env_r.k  # the same episodes were played on every env
    assert col.envstep == st["steps"]


def _device_cut(cfg, eps, n, n_ep, poll):
    """EpisodeSchedule + episode_segments over lockstep envs polled every `poll` iterations"""
    sched = EpisodeSchedule(n, n_ep)
    ends = [np.cumsum([len(e["action"]) for e in eps[i]]) - 1 for i in range(n)]
    seen = [0] * n
    it = 0
    pool = []
    while not sched.complete:
        it += poll
        batch = []
        for i in range(n):
            while seen[i] < len(eps[i]) and ends[i][seen[i]] < it:
                batch.append((i, len(eps[i][seen[i]]["action"]), eps[i][seen[i]]))
                seen[i] += 1
        for start, i, e in sched.take(batch):
            for itr, k, seg, pr, d in episode_segments(cfg, Discrete(A), e["obs"], e["action"], e["reward"], e["visits"],
                                                       e["value"], e["pred"], start, np.ones(A, np.int8), -1):
                pool.append((itr, i, k, seg, pr, d))
        assert it < 10 ** 6
    pool.sort(key=lambda x: x[:3])
    return [p[3] for p in pool], [{'priorities': p[4], 'done': p[5], 'unroll_plus_td_steps': cfg.num_unroll_steps +
                                   cfg.td_steps} for p in pool], sched


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("poll", [1, 4])
def test_device_cutter_matches_restatement(case, poll):
    n, n_ep, gsl, U, TD, fs, prio, ign = case
    rng = np.random.default_rng(7 + sum(case[:5]))
    eps = [[_episode(rng, L) for L in _lengths(rng, gsl)] for _ in range(n)]
    cfg = _cfg(gsl, U, TD, fs, prio, ign)
    segs, meta, sched = _device_cut(cfg, eps, n, n_ep, poll)
    # the restatement plays exactly the episodes the schedule counted
    played = [list(p) for p in sched.played]
    env_r = _Env(played)
    ref_segs, ref_meta, st = ref_collect(cfg, env_r, EpisodeForward(env_r), n_ep)
    assert env_r.k == [len(p) for p in played]
    _compare(segs, meta, ref_segs, ref_meta)


def test_schedule_hands_out_exactly_n_episode():
    rng = np.random.default_rng(3)
    for n, n_ep in [(4, 4), (4, 10), (8, 9), (1, 5)]:
        eps = [[_episode(rng, int(rng.integers(1, 30)), pred=False) for _ in range(12)] for _ in range(n)]
        cfg = _cfg(10, 5, 5, 1, False, False)
        segs, meta, sched = _device_cut(cfg, eps, n, n_ep, 3)
        assert sched.collected == n_ep == sum(len(p) for p in sched.played)
        assert all(len(p) >= 1 for p in sched.played)


def test_game_segment_surface():
    """GameSegment mirrors game_segment.py: get_obs window, is_full, store_search_stats zero-sum guard,
    pad_over bounds, game_segment_to_array ragged child visits"""
    from lightzero_amd.game_segment import GameSegment
    cfg = _cfg(3, 2, 2, 2, False, False)
    g = GameSegment(Discrete(A), 3, cfg)
    o0 = np.zeros(4, np.float32)
    g.reset([o0, o0])
    assert len(g.get_obs()) == 2 and not g.is_full()
    for t in range(3):
        g.store_search_stats([0, 0] if t == 0 else [1, 3], 0.5)
        g.append(np.int64(t % 2), np.full(4, t + 1, np.float32), 1.0, np.ones(2, np.int8), -1)
    assert g.is_full() and len(g) == 3
    assert g.child_visit_segment[0] == [0.0, 0.0] and g.child_visit_segment[1] == [0.25, 0.75]
    with pytest.raises(AssertionError):
        g.pad_over([o0] * 3, [], [], [])
    g.pad_over([o0], [1.0], [0.1, 0.2], [[1.0]])
    g.game_segment_to_array()
    assert g.child_visit_segment.dtype == object  # ragged
    assert g.obs_segment.shape == (6, 4) and g.reward_segment.shape == (4,)
    assert torch is not None


def test_device_path_routes_muzero_and_efficientzero_policies():
    """a DeviceEnvManager selects the device collector for MuZero and EfficientZero policies alike (the
    device search step picks the value-prefix / LSTM search from the model, efficientzero.py:538-656);
    collect_with_pure_policy keeps the host loop"""
    from lightzero_amd.envs import DeviceBreakoutEnvManager
    from lightzero_amd.policy import EfficientZeroCollectPolicy, MuZeroCollectPolicy
    cfg = policy_config(num_simulations=4, device='cpu',
                        model=dict(frame_stack_num=4, action_space_size=4, observation_shape=(4, 64, 64),
                                   image_channel=1, model_type='conv'))
    model = torch.nn.Linear(1, 1)  # (routing only: no forward)
    env = DeviceBreakoutEnvManager(4, seed=1)
    for cls, device_path in ((MuZeroCollectPolicy, True), (EfficientZeroCollectPolicy, True)):
        col = MuZeroCollector(env=env, policy=cls(cfg, model), policy_config=cfg)
        assert col._device_path(False) is device_path, cls.__name__
        assert col._device_path(True) is False  # collect_with_pure_policy: the host loop
