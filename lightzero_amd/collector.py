"""Device-resident collector for CartPole-v0 — the collector's fast mode.

Mirrors what MuZeroCollector.collect (lzero/worker/muzero_collector.py:399-705) does per env step
for a MuZero policy — stack the observation, run the collect-time search
(MuZeroPolicy._forward_collect, policy/muzero.py:617-690), select an action from the root visit
counts (select_action, policy/utils.py:515-539), step the env, append to the GameSegment
(game_segment.py:129-218) — with everything on the device: one HIP graph per env step holds
initial_inference, root preparation with Dirichlet noise, the fused search and the
`lzm_cartpole_collect_step` kernel (action sampling, recording, env physics, auto-reset, next
noise). The host only polls the finished-episode counters every `poll_every` steps.

Each env records its episodes into device slots (obs, action, reward, root visit COUNTS, root
value and, with `record_pred`, the root's predicted value for priorities). `collect(n_episode)`
returns whole episodes as GameSegment-shaped dicts; MuZeroCollector's device path
(lightzero_amd.worker.muzero_collector) cuts them into game_segment_length blocks with the
reference's rollover / pad_over / priorities (lightzero_amd.worker.segments). The env restates
gymnasium's CartPole equations (gymnasium is not installed: env parity unpinned); random streams
are Philox, not numpy's (the host-parity mode is MuZeroCollector over MuZeroCollectPolicy).
"""
import time
import weakref

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, ptr, stream_ptr
from .collect import DeviceSearchStep
from .trajectory import all_gather_packed, allreduce_stats, pack_episodes, unpack_episodes


class DeviceCollector:
    OBS_DIM = 4
    A = 2

    def __init__(self, model, env_num, num_simulations, device="cuda", max_episode_steps=200, episode_slots=8,
                 temperature=1.0, deterministic=False, noise_alpha=0.3, noise_weight=0.25, seed=0,
                 rng_mode="glibc", graph=True, poll_every=8, record_pred=False, support_scale=300):
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
        self.rec_visits = torch.zeros((n, E, T, A), dtype=torch.int32, device=dev)
        self.rec_value = torch.zeros((n, E, T), dtype=torch.float32, device=dev)
        self.rec_pred = torch.zeros((n, E, T), dtype=torch.float32, device=dev) if record_pred else None
        self._pred_transform = None
        if record_pred:
            from .scaling_transform import InverseScalarTransform
            self._pred_transform = InverseScalarTransform(support_scale, dev, True)
        self._epoch = 0
        self.ep_len = torch.zeros((n, E), dtype=torch.int32, device=dev)
        self.ep_count = torch.zeros(n, dtype=torch.int32, device=dev)
        me = weakref.ref(self)  # no collector <-> search-step reference cycle

        def epilogue(out):
            me()._env_step(out)

        self.search = DeviceSearchStep(model, n, self.S, [[0, 1]] * n, (4,), dev, noise_weight=noise_weight,
                                       seed=seed, rng_mode=rng_mode, graph=graph, epilogue=epilogue,
                                       support_scale=support_scale)
        self.search.build_graph()
        self.reset()

    def _env_step(self, out):
        pred = None
        if self._pred_transform is not None:  # predicted root value for priorities (muzero.py:667)
            pred = self._pred_transform(out["value_logits"]).reshape(-1)
        call("lzm_cartpole_collect_step", self.n, self.A, self.T, self.E, ptr(out["distributions"]),
             ptr(out["values"]), ptr(pred), ptr(self.state), ptr(self.steps), ptr(self.search.obs),
             ptr(self.search.noises), float(self.noise_alpha), float(self.temperature), int(self.deterministic),
             ptr(self.rec_obs), ptr(self.rec_action), ptr(self.rec_reward), ptr(self.rec_visits), ptr(self.rec_value),
             ptr(self.rec_pred), ptr(self.ep_len), ptr(self.ep_count), int(self.T), self.seed,
             ptr(self.search.step_counter), stream_ptr())

    def set_temperature(self, temperature, deterministic=None):
        """Change the action-selection temperature (policy_kwargs['temperature']); the captured step
        bakes it in, so a change re-captures the graph."""
        t = float(temperature)
        d = self.deterministic if deterministic is None else bool(deterministic)
        if t != self.temperature or d != self.deterministic:
            self.temperature, self.deterministic = t, d
            if self.search.graph is not None:
                # (capturing runs the step twice eagerly and zeroes the counter: keep the counter,
                # then start every env afresh)
                count = self.search.step_counter.clone()
                self.search.graph = None
                self.search.build_graph()
                self.search.step_counter.copy_(count)
                self.restart()

    def restart(self):
        """Every env to a fresh episode and the episode slots emptied, keeping the step counter (the
        Philox streams of later steps stay fresh); the resets draw from a new epoch of the seed."""
        self._epoch += 1
        self._reset_envs((self.seed + 0x9E3779B9 * self._epoch) & 0xFFFFFFFF)

    def reset(self):
        """All envs to a fresh episode; first root noise drawn on the host side of the stream."""
        self._epoch = 0
        self.envstep = 0
        self._reset_envs(self.seed)
        self.search.reset_seed_counter()

    def _reset_envs(self, seed):
        call("lzm_cartpole_reset", self.n, ptr(self.state), ptr(self.steps), ptr(self.search.obs), seed,
             stream_ptr())
        g = torch.Generator(device=self.dev).manual_seed(seed)
        conc = torch.full((self.n, self.A), self.noise_alpha, dtype=torch.float64, device=self.dev)
        gam = torch._standard_gamma(conc, generator=g) if hasattr(torch, "_standard_gamma") else None
        noise = (gam / gam.sum(dim=1, keepdim=True)).float() if gam is not None else torch.full_like(conc, 0.5).float()
        self.search.noises.copy_(noise)
        self.ep_count.zero_()
        self.ep_len.zero_()
        self._consumed = np.zeros(self.n, dtype=np.int64)
        self._gathered_at = getattr(self, "envstep", 0)

    def step(self):
        """One env step for every env (one graph replay)."""
        self.search.step()
        self.envstep += self.n

    def collect(self, n_episode, group=None):
        """Step until `n_episode` new episodes have finished on this rank; returns (episodes, stats).

        With an initialised torch.distributed process group of more than one rank (one collector
        per GPU, env-sharded), every rank's finished episodes are packed on its device and
        all-gathered (lightzero_amd.trajectory, RCCL over xGMI), and the step / episode / duration
        statistics are sum-reduced (muzero_collector.py:709-712): every rank returns the episodes
        of all ranks, each tagged with its `rank`."""
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        steps0 = self.envstep
        while True:
            for _ in range(self.poll_every):
                self.step()
            counts = self.ep_count.cpu().numpy().astype(np.int64)
            self.search.roots.tree.check_errors()  # (already synchronised) tie-break stream intact
            new = counts - self._consumed
            if (new >= self.E).any():  # the running episode reuses slot ep_count % E
                raise RuntimeError("episode slots overwritten before collection: raise episode_slots or lower "
                                   "poll_every")
            if new.sum() >= n_episode:
                break
        el = time.perf_counter() - t0
        return self._return(counts, self.envstep - steps0, el, group)

    def gather_finished(self, group=None):
        """The episodes finished since the last collect / gather, without stepping: packed on the
        device and, under a process group of more than one rank, all-gathered with the statistics
        sum-reduced (as collect does). Returns (episodes, stats)."""
        counts = self.ep_count.cpu().numpy().astype(np.int64)
        self.search.roots.tree.check_errors()
        if ((counts - self._consumed) >= self.E).any():  # the running episode reuses slot ep_count % E
            raise RuntimeError("episode slots overwritten before collection: raise episode_slots")
        steps = self.envstep - getattr(self, "_gathered_at", 0)
        return self._return(counts, steps, 0.0, group)

    def _return(self, counts, steps, el, group):
        packed, index = self._pack(counts)
        self._gathered_at = self.envstep
        world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        if world > 1:
            rank = dist.get_rank(group)
            blocks = all_gather_packed(packed, index, group)
            episodes = [e for r, (p, i) in enumerate(blocks) for e in unpack_episodes(p, i, self.OBS_DIM, self.A, r)]
            tot_steps, tot_eps, tot_secs = allreduce_stats(steps, len(index), el, self.dev, group)
        else:
            rank = 0
            episodes = unpack_episodes(packed.cpu().numpy(), index.numpy(), self.OBS_DIM, self.A)
            tot_steps, tot_eps, tot_secs = steps, len(episodes), el
        stats = dict(envstep=steps, seconds=el, env_steps_per_s=steps / el if el else None,
                     sims_per_s=steps * self.S / el if el else None,
                     episode_returns=[float(e["reward_segment"].sum()) for e in episodes], rank=rank, world=world,
                     total_envstep=tot_steps, total_episodes=tot_eps, total_duration=tot_secs)
        return episodes, stats

    def _pack(self, counts):
        """the episodes finished since the last collect, packed on the device (trajectory.pack_episodes)"""
        ln = self.ep_len.cpu().numpy()
        todo = []
        for i in range(self.n):
            for k in range(int(self._consumed[i]), int(counts[i])):
                e = k % self.E
                todo.append((i, e, int(ln[i, e])))
            self._consumed[i] = counts[i]
        return pack_episodes(self.rec_obs, self.rec_action, self.rec_reward, self.rec_visits, self.rec_value, todo,
                             self.rec_pred)

    def pull_new(self):
        """The episodes finished since the last pull, on the host (one device pack + one copy):
        (env_id, L, episode dict) in env order, each env's episodes in finishing order."""
        counts = self.ep_count.cpu().numpy().astype(np.int64)
        if ((counts - self._consumed) >= self.E).any():  # the running episode reuses slot ep_count % E
            raise RuntimeError("episode slots overwritten before collection: raise episode_slots or lower poll_every")
        packed, index = self._pack(counts)
        return unpack_episodes(packed.cpu().numpy(), index.numpy(), self.OBS_DIM, self.A)
