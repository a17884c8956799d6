"""Device-resident collector for CartPole-v0.

Mirrors what MuZeroCollector.collect (lzero/worker/muzero_collector.py:399-705) does per env step
for a MuZero policy — stack the observation, run the collect-time search
(MuZeroPolicy._forward_collect, policy/muzero.py:617-690), select an action from the root visit
counts (select_action, policy/utils.py:515-539), step the env, append to the GameSegment
(game_segment.py:129-218) — with everything on the device: one HIP graph per env step holds
initial_inference, root preparation with Dirichlet noise, the fused search and the
`lzm_cartpole_collect_step` kernel (action sampling, recording, env physics, auto-reset, next
noise). The host only polls the finished-episode counters every `poll_every` steps.

Episodes are returned as GameSegment-shaped dicts (obs_segment, action_segment, reward_segment,
child_visit_segment, root_value_segment, to_play_segment, action_mask_segment). Cutting them into
game_segment_length blocks with padding (GameSegment.pad_over) belongs to the replay buffer and is
out of scope. The env restates gymnasium's CartPole equations (gymnasium is not
installed: env parity unpinned); random streams are Philox, not numpy's.
"""
import time
import weakref

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr
from .collect import DeviceSearchStep


class DeviceCollector:
    OBS_DIM = 4
    A = 2

    def __init__(self, model, env_num, num_simulations, device="cuda", max_episode_steps=200, episode_slots=8,
                 temperature=1.0, deterministic=False, noise_alpha=0.3, noise_weight=0.25, seed=0,
                 rng_mode="glibc", graph=True, poll_every=8):
        _lib.require_gpu()
        self.n, self.S = int(env_num), int(num_simulations)
        self.dev = torch.device(device)
        self.T = int(max_episode_steps)
        self.E = int(episode_slots)
        self.temperature, self.deterministic = float(temperature), bool(deterministic)
        self.noise_alpha = float(noise_alpha)
        self.seed = int(seed) & 0xFFFFFFFF
        self.poll_every = int(poll_every)
        n, A, T, E, dev = self.n, self.A, self.T, self.E, self.dev
        self.state = torch.zeros((n, 4), dtype=torch.float64, device=dev)
        self.steps = torch.zeros(n, dtype=torch.int32, device=dev)
        self.rec_obs = torch.zeros((n, E, T + 1, 4), dtype=torch.float32, device=dev)
        self.rec_action = torch.zeros((n, E, T), dtype=torch.int32, device=dev)
        self.rec_reward = torch.zeros((n, E, T), dtype=torch.float32, device=dev)
        self.rec_child = torch.zeros((n, E, T, A), dtype=torch.float32, device=dev)
        self.rec_value = torch.zeros((n, E, T), dtype=torch.float32, device=dev)
        self.ep_len = torch.zeros((n, E), dtype=torch.int32, device=dev)
        self.ep_count = torch.zeros(n, dtype=torch.int32, device=dev)
        me = weakref.ref(self)  # no collector <-> search-step reference cycle

        def epilogue(out):
            me()._env_step(out)

        self.search = DeviceSearchStep(model, n, self.S, [[0, 1]] * n, (4,), dev, noise_weight=noise_weight,
                                       seed=seed, rng_mode=rng_mode, graph=graph, epilogue=epilogue)
        self.search.build_graph()
        self.reset()

    def _env_step(self, out):
        call("lzm_cartpole_collect_step", self.n, self.A, self.T, self.E, ptr(out["distributions"]),
             ptr(out["values"]), ptr(self.state), ptr(self.steps), ptr(self.search.obs), ptr(self.search.noises),
             float(self.noise_alpha), float(self.temperature), int(self.deterministic), ptr(self.rec_obs),
             ptr(self.rec_action), ptr(self.rec_reward), ptr(self.rec_child), ptr(self.rec_value), ptr(self.ep_len),
             ptr(self.ep_count), int(self.T), self.seed, ptr(self.search.step_counter), stream_ptr())

    def reset(self):
        """All envs to a fresh episode; first root noise drawn on the host side of the stream."""
        call("lzm_cartpole_reset", self.n, ptr(self.state), ptr(self.steps), ptr(self.search.obs), self.seed,
             stream_ptr())
        g = torch.Generator(device=self.dev).manual_seed(self.seed)
        conc = torch.full((self.n, self.A), self.noise_alpha, dtype=torch.float64, device=self.dev)
        gam = torch._standard_gamma(conc, generator=g) if hasattr(torch, "_standard_gamma") else None
        noise = (gam / gam.sum(dim=1, keepdim=True)).float() if gam is not None else torch.full_like(conc, 0.5).float()
        self.search.noises.copy_(noise)
        self.ep_count.zero_()
        self.ep_len.zero_()
        self.search.reset_seed_counter()
        self._consumed = np.zeros(self.n, dtype=np.int64)
        self.envstep = 0

    def step(self):
        """One env step for every env (one graph replay)."""
        self.search.step()
        self.envstep += self.n

    def collect(self, n_episode):
        """Step until `n_episode` new episodes have finished; returns (episodes, stats)."""
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        steps0 = self.envstep
        while True:
            for _ in range(self.poll_every):
                self.step()
            counts = self.ep_count.cpu().numpy().astype(np.int64)
            new = counts - self._consumed
            if (new >= self.E).any():  # the running episode reuses slot ep_count % E
                raise RuntimeError("episode slots overwritten before collection: raise episode_slots or lower "
                                   "poll_every")
            if new.sum() >= n_episode:
                break
        el = time.perf_counter() - t0
        episodes = self._gather(counts)
        steps = self.envstep - steps0
        stats = dict(envstep=steps, seconds=el, env_steps_per_s=steps / el, sims_per_s=steps * self.S / el,
                     episode_returns=[float(e["reward_segment"].sum()) for e in episodes])
        return episodes, stats

    def _gather(self, counts):
        ln = self.ep_len.cpu().numpy()
        obs, act = self.rec_obs.cpu().numpy(), self.rec_action.cpu().numpy()
        rew, child, val = self.rec_reward.cpu().numpy(), self.rec_child.cpu().numpy(), self.rec_value.cpu().numpy()
        eps = []
        for i in range(self.n):
            for k in range(int(self._consumed[i]), int(counts[i])):
                e = k % self.E
                L = int(ln[i, e])
                eps.append(dict(env_id=i, obs_segment=obs[i, e, :L + 1].copy(), action_segment=act[i, e, :L].copy(),
                                reward_segment=rew[i, e, :L].copy(), child_visit_segment=child[i, e, :L].copy(),
                                root_value_segment=val[i, e, :L].copy(), to_play_segment=np.full(L, -1, np.int32),
                                action_mask_segment=np.ones((L, self.A), np.int8)))
            self._consumed[i] = counts[i]
        return eps
