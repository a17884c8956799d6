"""Cutting finished episodes into GameSegments, vectorised, for the device collector path.

MuZeroCollector.collect (lzero/worker/muzero_collector.py:399-705) builds segments step by step:
every `game_segment_length` transitions the running segment is full, the previous one is padded
with the new one's first frames / rewards / root values / visit distributions
(`pad_and_save_last_trajectory`, :229-301) and saved, and at the end of an episode the last two
are padded / saved (:612-632). The device collector records whole episodes on the GPU, so here
the same segments — contents, `done` flags, priorities and their position in the collector's
pool — are computed from one episode's arrays at once:

  segment j covers transitions [s_j, s_j + n_j), s_j = j * gsl, n_j = min(gsl, L - s_j); its
  observations start with the frame-stack window ending at o_{s_j} (the reset frame repeated at the
  episode start); the pad from segment j + 1 (n' of its transitions) adds
  o_{s_{j+1}+1 .. +min(U, n')}, visit distributions [: min(U, n')], rewards [: min(U + TD - 1, n')]
  and root values [: min(U + TD, n')]; a full last segment is padded with the empty segment that
  follows it, a partial last segment is saved unpadded.

Save order key (iteration, env_id, k): the collector appends to its pool while it walks one
iteration's timesteps in env order; within an env the rollover save comes before the two end-of-
episode saves.
"""
import numpy as np

from ..game_segment import GameSegment


def episode_segments(cfg, action_space, obs, action, reward, visits, root_value, pred_value, start_iter,
                     action_mask, to_play):
    """One finished episode -> [(iteration, k, GameSegment, priorities, done)].

    obs [L + 1, ...] (o_0 the reset frame), action [L] int, reward [L], visits [L, A] int
    (legal-order counts), root_value [L], pred_value [L] or None (priorities need it),
    start_iter: the collector iteration of transition 0."""
    L = int(len(action))
    gsl = int(cfg.game_segment_length)
    U, TD = int(cfg.num_unroll_steps), int(cfg.td_steps)
    fs = int(cfg.model.frame_stack_num)
    ignore_done = bool(cfg.get('ignore_done', False))
    use_priority = bool(cfg.get('use_priority', False))
    tot = visits.sum(axis=1, keepdims=True).astype(np.float64)
    tot[tot == 0] = 1e-6
    child = visits.astype(np.float64) / tot  # store_search_stats: visit / sum, in float64
    rew = np.asarray(reward, np.float64)
    val = np.asarray(root_value, np.float32).astype(np.float64)
    act = np.asarray(action, np.int64)
    # frame-stack window: fs copies of o_0, then o_1 .. o_L
    frames = np.concatenate([np.repeat(obs[:1], fs - 1, axis=0), obs], axis=0) if fs > 1 else obs
    m = -(-L // gsl)  # non-empty segments
    last_full = L % gsl == 0
    end_iter = start_iter + L - 1
    out = []
    for j in range(m):
        s = j * gsl
        n = min(gsl, L - s)
        # the next segment as it stands when this one is padded (empty after a full last segment)
        s2 = s + gsl
        n2 = min(gsl, L - s2) if s2 < L else 0
        padded = j < m - 1 or last_full
        po = min(U, n2) if padded else 0
        o = frames[s:s + fs + n]  # window (fs) + o_{s+1 .. s+n}
        if po:
            o = np.concatenate([o, obs[s2 + 1:s2 + 1 + po]], axis=0)
        r = rew[s:s + n]
        v = val[s:s + n]
        c = child[s:s + n]
        if padded:
            r = np.concatenate([r, rew[s2:s2 + min(U + TD - 1, n2)]])
            v = np.concatenate([v, val[s2:s2 + min(U + TD, n2)]])
            c = np.concatenate([c, child[s2:s2 + min(U, n2)]], axis=0)
        seg = GameSegment.from_arrays(action_space, gsl, cfg, o, act[s:s + n], r, c, v,
                                      np.repeat(np.asarray(action_mask)[None], n, axis=0), np.full(n, to_play, np.int64))
        prio = None
        if use_priority:
            prio = np.abs(np.asarray(pred_value[s:s + n], np.float32) - np.asarray(root_value[s:s + n], np.float32)) \
                + np.float32(1e-6)
        if j < m - 1:
            # saved when segment j + 1 fills (rollover save, k = 0) or at the episode's end (k = 1)
            full_next = n2 == gsl
            it = start_iter + s2 + gsl - 1 if full_next else end_iter
            k = 0 if full_next else 1
        else:
            # the last non-empty segment: padded with the empty one (k = 1) if full, else saved as the
            # current segment (k = 2), both at the episode's end
            it, k = end_iter, (1 if last_full else 2)
        done = (not ignore_done) and it == end_iter
        out.append((it, k, seg, prio, done))
    return out


class EpisodeSchedule:
    """The reference collector's episode accounting replayed on lockstep device envs.

    In MuZeroCollector.collect every env starts one episode; when one finishes it is handed a new
    one while `remain_episode` lasts (n_episode > env_num), lower env ids first within an
    iteration (the ready-set union), otherwise it sits idle; the call returns once n_episode
    episodes have finished. The device steps every env every iteration, so episodes an env plays
    past its share are dropped here. Feed `finished` in poll batches (each env's episodes in order,
    episodes starting back to back from iteration 0); `take` returns the counted ones with their
    start iteration, in the order the reference finishes them."""

    def __init__(self, env_num, n_episode):
        self.n, self.n_episode = int(env_num), int(n_episode)
        self.assigned = np.ones(self.n, np.int64)
        self.finished = np.zeros(self.n, np.int64)
        self.pos = np.zeros(self.n, np.int64)
        self.remain = self.n_episode - self.n
        self.collected = 0
        self.played = [[] for _ in range(self.n)]  # counted episodes per env, in order

    @property
    def complete(self):
        return self.collected >= self.n_episode

    def take(self, finished):
        """finished: [(env_id, L, payload)] of one poll -> [(start_iter, env_id, payload)] counted"""
        ev = []
        for i, L, payload in finished:
            ev.append((int(self.pos[i]) + int(L) - 1, int(i), int(L), payload))
            self.pos[i] += int(L)
        out = []
        for end, i, L, payload in sorted(ev, key=lambda x: (x[0], x[1])):
            if self.finished[i] >= self.assigned[i] or self.complete:
                continue  # idle in the reference's schedule
            self.finished[i] += 1
            self.collected += 1
            self.played[i].append(payload)
            out.append((end - L + 1, i, payload))
            if self.n_episode > self.n and self.remain > 0:
                self.assigned[i] += 1
                self.remain -= 1
        return out
