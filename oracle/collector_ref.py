"""Host restatement of LightZero's collect loop — TEST INFRASTRUCTURE ONLY.

Imported by tests/ only, as the checker for lightzero_amd.worker.MuZeroCollector (host loop and
device path) and lightzero_amd.policy.MuZeroCollectPolicy. Never imported by the product.

Restates, from the reference (paths relative to /root/reference):
  lzero/worker/muzero_collector.py:305-705     collect(): ready-env bookkeeping, step processing,
                                              rollover, end-of-episode saves, pool order
  lzero/worker/muzero_collector.py:200-301     _compute_priorities, pad_and_save_last_trajectory
  lzero/mcts/buffer/game_segment.py:129-294    append, store_search_stats, pad_over, to_array
  lzero/policy/muzero.py:617-740               _forward_collect (noise, roots, search, select_action)
  lzero/policy/muzero.py:783-867               _forward_eval (prepare_no_noise, search, argmax)
  lzero/policy/efficientzero.py:538-656        _forward_collect with the value-prefix tree (is_reset)
  lzero/policy/utils.py:515-539                select_action

`replay_forward` is _forward_collect with the search done by the oracle tree (oracle.OracleTree,
the pinned ctree restatement) fed the network outputs a GPU run recorded, and numpy drawing the
noise and the actions in the reference's order — so on the same numpy seed it must reproduce the
GPU collector's actions, visit counts and root values bit for bit.
"""
import copy
from collections import deque

import numpy as np
from scipy.stats import entropy

from oracle.oracle import OracleTree

PB_C_BASE, PB_C_INIT, DISC, VDM = 19652, np.float32(1.25), np.float32(0.997), np.float32(0.01)


class Seg:
    """game_segment.py's GameSegment, list form, restated for the checker"""

    def __init__(self, cfg, init_frames):
        self.cfg = cfg
        self.obs = [copy.deepcopy(f) for f in init_frames]
        self.act, self.rew, self.cv, self.rv, self.mask, self.tp = [], [], [], [], [], []

    def stacked_obs(self):
        fs = self.cfg.model.frame_stack_num
        t = len(self.rew)
        assert len(self.obs) - fs == t
        return self.obs[t:t + fs]

    def record(self, visits, value, action, next_obs, reward, mask, to_play):
        s = sum(visits) or 1e-6
        self.cv.append([v / s for v in visits])
        self.rv.append(value)
        self.act.append(action)
        self.obs.append(next_obs)
        self.rew.append(reward)
        self.mask.append(mask)
        self.tp.append(to_play)

    def full(self):
        return len(self.act) >= self.cfg.game_segment_length

    def pad_from(self, nxt):
        fs, U, TD = self.cfg.model.frame_stack_num, self.cfg.num_unroll_steps, self.cfg.td_steps
        self.obs += [copy.deepcopy(o) for o in nxt.obs[fs:fs + U]]
        self.rew += nxt.rew[:U + TD - 1]
        self.rv += nxt.rv[:U + TD]
        self.cv += nxt.cv[:U]

    def arrays(self):
        return dict(obs_segment=np.array(self.obs), action_segment=np.array(self.act),
                    reward_segment=np.array(self.rew), child_visit_segment=np.array(self.cv),
                    root_value_segment=np.array(self.rv), action_mask_segment=np.array(self.mask),
                    to_play_segment=np.array(self.tp))


def _priorities(cfg, preds, searched):
    if not cfg.use_priority:
        return None
    p = np.array(preds, dtype=np.float64).astype(np.float32).reshape(-1)
    s = np.array(searched, dtype=np.float64).astype(np.float32).reshape(-1)
    return np.abs(p - s) + 1e-6


def ref_collect(cfg, env, forward, n_episode, temperature=1.0, epsilon=0.0):
    """muzero_collector.py:305-705 over an env manager (ready_obs / step) and a forward function
    with _forward_collect's signature. Returns (segments as dicts of arrays, meta list, stats)."""
    fs = cfg.model.frame_stack_num
    n = env.env_num
    obs0 = env.ready_obs
    mask = {i: np.asarray(obs0[i]['action_mask']) for i in range(n)}
    tplay = {i: np.array(obs0[i]['to_play']) for i in range(n)}
    win = {i: deque([np.asarray(obs0[i]['observation'])] * fs, maxlen=fs) for i in range(n)}
    cur = {i: Seg(cfg, win[i]) for i in range(n)}
    prev = {i: None for i in range(n)}
    prev_prio = {i: None for i in range(n)}
    preds = {i: [] for i in range(n)}
    srch = {i: [] for i in range(n)}
    dones = np.zeros(n, bool)
    pool = []
    ready, remain, finished, steps = set(), n_episode, 0, 0

    def save_prev(i):
        prev[i].pad_from(cur[i])
        pool.append((prev[i].arrays(), prev_prio[i], bool(dones[i])))
        prev[i] = prev_prio[i] = None

    def admit(avail):
        nonlocal ready, remain
        ready = ready.union(set(list(avail)[:remain]))
        remain -= min(len(avail), remain)

    while True:
        admit(set(env.ready_obs.keys()).difference(ready))
        order = list(ready)
        data = np.array([cur[i].stacked_obs() for i in order]).reshape(len(order), -1)
        out = forward(data, [mask[i] for i in order], temperature, [tplay[i] for i in order], epsilon, order)
        ts = env.step({i: out[i]['action'] for i in order})
        for i, t in ts.items():
            o = out[i]
            cur[i].record(o['visit_count_distributions'], o['searched_value'], o['action'],
                          np.asarray(t.obs['observation']), t.reward, mask[i], tplay[i])
            mask[i], tplay[i] = np.asarray(t.obs['action_mask']), np.array(t.obs['to_play'])
            dones[i] = False if cfg.ignore_done else t.done
            if cfg.use_priority:
                preds[i].append(o['predicted_value'])
                srch[i].append(o['searched_value'])
            win[i].append(np.asarray(t.obs['observation']))
            if cur[i].full():
                if prev[i] is not None:
                    save_prev(i)
                prev[i], prev_prio[i] = cur[i], _priorities(cfg, preds[i], srch[i])
                preds[i], srch[i] = [], []
                cur[i] = Seg(cfg, win[i])
            steps += 1
            if not t.done:
                continue
            finished += 1
            if prev[i] is not None:
                save_prev(i)
            pr = _priorities(cfg, preds[i], srch[i])
            if cur[i].rew:
                pool.append((cur[i].arrays(), pr, bool(dones[i])))
            if n_episode > n:
                obs_r = env.ready_obs
                admit(set(obs_r.keys()).difference(ready))
                mask[i], tplay[i] = np.asarray(obs_r[i]['action_mask']), np.array(obs_r[i]['to_play'])
                win[i] = deque([obs_r[i]['observation']] * fs, maxlen=fs)
                cur[i] = Seg(cfg, win[i])
                prev[i] = prev_prio[i] = None
            preds[i], srch[i] = [], []
            ready.remove(i)
        if finished >= n_episode:
            meta = [{'priorities': p, 'done': d, 'unroll_plus_td_steps': cfg.num_unroll_steps + cfg.td_steps}
                    for _, p, d in pool]
            return [s for s, _, _ in pool], meta, dict(steps=steps, episodes=finished)


def ref_select_action(visits, temperature, deterministic):
    pw = [v ** (1 / temperature) for v in visits]
    tot = sum(pw)
    probs = [x / tot for x in pw]
    pos = np.argmax(visits) if deterministic else np.random.choice(len(visits), p=probs)
    return pos, entropy(probs, base=2)


class ReplayForward:
    """_forward_collect (muzero.py:617-740) with the oracle tree replaying a GPU run's recorded
    search (MuZeroCollectPolicy.records, one per forward) and numpy drawing noise and actions.
    Every request of the oracle tree is checked against the recorded one."""

    def __init__(self, cfg, records):
        self.cfg, self.records, self.k = cfg, records, 0
        self.mismatch = []
        # EfficientZeroPolicy (efficientzero.py:538-656): the value-prefix tree, is_reset every
        # lstm_horizon_len levels (mcts_ctree.py:810-816)
        self.ez = cfg.get('type', 'muzero') == 'efficientzero'

    def _tree_search(self, rec, B, legal, noises, to_play):
        """the oracle tree replaying the GPU run's recorded search; returns (distributions, values)"""
        cfg = self.cfg
        A = max(len(l) for l in legal)
        S = cfg.num_simulations
        t = OracleTree(B, A, S, ez=self.ez)
        lg = np.full((B, A), -1, np.int32)
        for j, l in enumerate(legal):
            lg[j, :len(l)] = l
        t.set_legal(lg, np.array([len(l) for l in legal], np.int32))
        t.set_delta(VDM)
        nz = None
        if noises is not None:
            nz = np.zeros((B, A), np.float32)
            for j, z in enumerate(noises):
                nz[j, :len(z)] = z
        tp = np.array([int(x) for x in to_play], np.int32)
        weight = np.float32(cfg.root_noise_weight) if noises is not None else np.float32(0.0)
        t.prepare(weight, nz, np.asarray(rec.get('reward_roots', np.zeros(B)), np.float32), rec['root_logits'], tp)
        sr = rec['search']
        horizon = int(cfg.get('lstm_horizon_len', 5))
        for s in range(S):
            x, y, a, vtp, slen = t.traverse(PB_C_BASE, PB_C_INIT, DISC, int(sr['seeds'][s]), tp)
            if not (np.array_equal(x, sr['x'][s]) and np.array_equal(a, sr['action'][s])
                    and np.array_equal(slen, sr['search_len'][s])):
                self.mismatch.append((self.k - 1, 'request', s))
            is_reset = (slen % horizon == 0).astype(np.int32) if self.ez else None
            t.backprop(s + 1, DISC, sr['decoded'][s][:, 0], sr['decoded'][s][:, 1], sr['policy_logits'][s], vtp,
                       is_reset)
        return t.distributions(), t.values()

    def _check_data(self, data, rec):
        if not np.array_equal(np.asarray(data, np.float32).reshape(-1), np.asarray(rec['data'], np.float32).reshape(-1)):
            self.mismatch.append((self.k - 1, 'observations'))

    def eval(self, data, action_mask, to_play, ready_env_id):
        """_forward_eval (muzero.py:783-867): prepare_no_noise, the search, argmax (no draw)"""
        rec = self.records[self.k]
        self.k += 1
        B = len(ready_env_id)
        self._check_data(data, rec)
        legal = [[a for a, m in enumerate(action_mask[j]) if m == 1] for j in range(B)]
        dist, vals = self._tree_search(rec, B, legal, None, to_play)
        out = {}
        for j, env_id in enumerate(ready_env_id):
            d = [int(v) for v in dist[j][:len(legal[j])]]
            pos, ent = ref_select_action(d, 1.0, True)
            out[env_id] = {'action': np.where(np.asarray(action_mask[j]) == 1.0)[0][pos],
                           'visit_count_distributions': d, 'visit_count_distribution_entropy': ent,
                           'searched_value': float(vals[j]), 'predicted_value': rec['pred_values'][j]}
        return out

    def __call__(self, data, action_mask, temperature, to_play, epsilon, ready_env_id):
        cfg = self.cfg
        rec = self.records[self.k]
        self.k += 1
        B = len(ready_env_id)
        assert B == len(rec['root_logits']), (f"forward {self.k - 1}: {B} ready envs, the GPU run had "
                                              f"{len(rec['root_logits'])} (mismatches so far: {self.mismatch[:5]})")
        self._check_data(data, rec)
        legal = [[a for a, m in enumerate(action_mask[j]) if m == 1] for j in range(B)]
        noises = [np.random.dirichlet([cfg.root_dirichlet_alpha] * int(sum(action_mask[j]))).astype(np.float32)
                  .tolist() for j in range(B)]
        if noises != rec['noises']:
            self.mismatch.append((self.k - 1, 'noises'))
        dist, vals = self._tree_search(rec, B, legal, noises, to_play)
        out = {}
        for j, env_id in enumerate(ready_env_id):
            d = [int(v) for v in dist[j][:len(legal[j])]]
            pos, ent = ref_select_action(d, temperature, cfg.eps.eps_greedy_exploration_in_collect)
            out[env_id] = {'action': np.where(np.asarray(action_mask[j]) == 1.0)[0][pos],
                           'visit_count_distributions': d, 'visit_count_distribution_entropy': ent,
                           'searched_value': float(vals[j]), 'predicted_value': rec['pred_values'][j]}
        return out


class EpisodeEnv:
    """An env manager that replays recorded episodes env by env (obs, rewards, done at the end;
    the next episode's first frame after a done), for checking segment cutting on fixed data."""

    def __init__(self, episodes_per_env):
        self.eps = episodes_per_env
        self.env_num = len(episodes_per_env)
        self.k = [0] * self.env_num   # episode index
        self.t = [0] * self.env_num   # step within it
        self._ready = {i: self._obs(i, 0) for i in range(self.env_num)}

    def _obs(self, i, t):
        e = self.eps[i][self.k[i]]
        return {'observation': e['obs'][t], 'action_mask': np.ones(e['visits'].shape[1], np.int8), 'to_play': -1}

    @property
    def ready_obs(self):
        return dict(self._ready)

    def step(self, actions):
        out = {}
        for i in sorted(actions):
            e = self.eps[i][self.k[i]]
            t = self.t[i]
            L = len(e['action'])
            done = t + 1 == L
            obs = self._obs(i, t + 1)

            class TS:
                pass
            ts = TS()
            ts.obs, ts.reward, ts.done = obs, float(e['reward'][t]), done
            ts.info = {'eval_episode_return': float(np.sum(e['reward']))} if done else {}
            out[i] = ts
            if done:
                self.k[i] += 1
                self.t[i] = 0
                self._ready[i] = self._obs(i, 0) if self.k[i] < len(self.eps[i]) else obs
            else:
                self.t[i] = t + 1
                self._ready[i] = obs
        return out


class EpisodeForward:
    """A forward that replays the recorded search outputs of EpisodeEnv's episodes"""

    def __init__(self, env):
        self.env = env

    def __call__(self, data, action_mask, temperature, to_play, epsilon, ready_env_id):
        out = {}
        for i in ready_env_id:
            e = self.env.eps[i][self.env.k[i]]
            t = self.env.t[i]
            d = [int(v) for v in e['visits'][t]]
            out[i] = {'action': np.int64(e['action'][t]), 'visit_count_distributions': d,
                      'visit_count_distribution_entropy': ref_select_action(d, temperature, True)[1] if sum(d) else 0.0,
                      'searched_value': float(np.float32(e['value'][t])),
                      'predicted_value': None if e.get('pred') is None else np.array([e['pred'][t]], np.float32)}
        return out
