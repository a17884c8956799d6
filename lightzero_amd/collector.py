"""Device-resident collector — the collector's fast mode.

Mirrors what MuZeroCollector.collect (lzero/worker/muzero_collector.py:399-705) does per env step
for a MuZero or EfficientZero policy — stack the observation, run the collect-time search
(MuZeroPolicy._forward_collect, policy/muzero.py:617-690; EfficientZeroPolicy._forward_collect,
policy/efficientzero.py:538-656, whose roots carry the value prefix and the LSTM state: the model picks
the search, DeviceSearchStep), select an action from the root visit
counts (select_action, policy/utils.py:515-539), step the env, append to the GameSegment
(game_segment.py:129-218) — with everything on the device: one HIP graph per env step holds
initial_inference, root preparation with Dirichlet noise, the search and the env's collect kernel
(action sampling, recording, env step, auto-reset, next noise). The host only polls the
finished-episode counters every `poll_every` steps.

Two device envs (DEVICE_ENVS):
- "cartpole": CartPole-v0 for config 2 (MuZeroModelMLP; one thread per env, lzm_collect.h);
  gymnasium's equations restated (gymnasium absent: env parity unpinned);
- "breakout": the Atari image path of config 5 (conv MuZeroModel, 4 x 64 x 64 stacked grey frames, 4
  actions; one workgroup per env, lzm_atari.h) — a stand-in game with Breakout's action set and frame
  format, since ALE is not installed (env parity unpinned; the frames, recording and trajectory sizes
  have the real shape);
- "pong": config 3's image path (conv EfficientZeroModel: the one-launch EfficientZero search with the
  reward LSTM in the same captured step; 6 actions) with a Pong stand-in game on the same kernel.

Each env records its episodes into device slots: one frame per step (the env's observation for
CartPole, the newest u8 grey frame for Atari — GameSegment stores one frame per step and stacks
frame_stack_num of them), action, reward, root visit COUNTS, root value and, with `record_pred`, the
root's predicted value for priorities. `collect(n_episode)` returns whole episodes as
GameSegment-shaped dicts, `collect_blocks` / `gather_blocks` the packed TrajBlocks (device packing:
lzm_episodes_scan / lzm_episodes_pack, one 24-byte read-back); MuZeroCollector's device path
(lightzero_amd.worker.muzero_collector) cuts episodes into game_segment_length blocks with the
reference's rollover / pad_over / priorities (lightzero_amd.worker.segments). Random streams are
Philox, not numpy's (the host-parity mode is MuZeroCollector over MuZeroCollectPolicy).
"""
import time
import weakref

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, ptr, stream_ptr
from .collect import DeviceSearchStep
from .trajectory import TrajBlock, all_gather_packed, allreduce_stats, gather_packed, scalar_width, unpack_episodes, \
    wire_bytes


class CartPoleDevice:
    """CartPole-v0 on the device (lzm_cartpole_*: one thread per env)."""
    name = "CartPole-v0"
    A = 2
    obs_shape = (4,)            # the model's observation
    frame_shape = (4,)          # one recorded observation per step
    frame_dtype = torch.float32
    frame_scale = 1.0
    frame_stack = 1
    support_scale = 300

    def __init__(self, n, dev):
        self.n = n
        self.state = torch.zeros((n, 4), dtype=torch.float64, device=dev)
        self.steps = torch.zeros(n, dtype=torch.int32, device=dev)

    def reset(self, obs, seed):
        call("lzm_cartpole_reset", self.n, ptr(self.state), ptr(self.steps), ptr(obs), seed, stream_ptr())

    def collect_step(self, c, out, pred):
        call("lzm_cartpole_collect_step", c.n, self.A, c.T, c.E, ptr(out["distributions"]), ptr(out["values"]),
             ptr(pred), ptr(self.state), ptr(self.steps), ptr(c.search.obs), ptr(c.search.noises),
             float(c.noise_alpha), float(c.temperature), int(c.deterministic), ptr(c.rec_frames),
             ptr(c.rec_action), ptr(c.rec_reward), ptr(c.rec_visits), ptr(c.rec_value), ptr(c.rec_pred),
             ptr(c.ep_len), ptr(c.ep_count), ptr(c.ep_return), int(c.T), c.seed, ptr(c.search.step_counter),
             stream_ptr())


class BreakoutDevice:
    """The Atari image env of config 5 on the device (lzm_atari_*: one workgroup per env): Breakout's
    minimal action set {NOOP, FIRE, RIGHT, LEFT}, grey 64 x 64 frames (u8 recorded, / 255 for the
    model), frame_stack_num 4, clipped rewards, one life per episode. A stand-in game (ALE absent)."""
    name = "Breakout (stand-in, ALE absent)"
    A = 4
    obs_shape = (4, 64, 64)
    frame_shape = (1, 64, 64)
    frame_dtype = torch.uint8
    frame_scale = 1.0 / 255.0
    frame_stack = 4
    support_scale = 300

    def __init__(self, n, dev):
        self.n = n
        self.state = torch.zeros((n, 16), dtype=torch.int32, device=dev)
        self.steps = torch.zeros(n, dtype=torch.int32, device=dev)
        self.cur = torch.zeros((n, 64 * 64), dtype=torch.uint8, device=dev)

    def reset(self, obs, seed):
        call("lzm_atari_reset", self.n, ptr(self.state), ptr(self.steps), ptr(self.cur), ptr(obs), seed, stream_ptr())

    def collect_step(self, c, out, pred):
        call("lzm_atari_collect_step", c.n, self.A, c.T, c.E, ptr(out["distributions"]), ptr(out["values"]),
             ptr(pred), ptr(self.state), ptr(self.steps), ptr(self.cur), ptr(c.search.obs), ptr(c.search.noises),
             float(c.noise_alpha), float(c.temperature), int(c.deterministic), ptr(c.rec_frames),
             ptr(c.rec_action), ptr(c.rec_reward), ptr(c.rec_visits), ptr(c.rec_value), ptr(c.rec_pred),
             ptr(c.ep_len), ptr(c.ep_count), ptr(c.ep_return), int(c.T), c.seed, ptr(c.search.step_counter),
             stream_ptr())


class PongDevice(BreakoutDevice):
    """Config 3's Atari image env on the device (lzm_pong_*, the same collect kernel as Breakout's with the Pong
    stand-in game, csrc/lzm_atari.h): Pong's minimal action set {NOOP, FIRE, RIGHT (up), LEFT (down), RIGHTFIRE,
    LEFTFIRE}, the agent's paddle on the right against a scripted opponent, +1 / -1 per point, 21 points end the
    episode, grey 64 x 64 frames, frame_stack_num 4. A stand-in game (ALE absent); EfficientZero's value support
    (scale 50: atari_efficientzero_config.py)."""
    name = "Pong (stand-in, ALE absent)"
    A = 6
    support_scale = 50

    def reset(self, obs, seed):
        call("lzm_pong_reset", self.n, ptr(self.state), ptr(self.steps), ptr(self.cur), ptr(obs), seed, stream_ptr())

    def collect_step(self, c, out, pred):
        call("lzm_pong_collect_step", c.n, self.A, c.T, c.E, ptr(out["distributions"]), ptr(out["values"]),
             ptr(pred), ptr(self.state), ptr(self.steps), ptr(self.cur), ptr(c.search.obs), ptr(c.search.noises),
             float(c.noise_alpha), float(c.temperature), int(c.deterministic), ptr(c.rec_frames),
             ptr(c.rec_action), ptr(c.rec_reward), ptr(c.rec_visits), ptr(c.rec_value), ptr(c.rec_pred),
             ptr(c.ep_len), ptr(c.ep_count), ptr(c.ep_return), int(c.T), c.seed, ptr(c.search.step_counter),
             stream_ptr())


DEVICE_ENVS = {"cartpole": CartPoleDevice, "breakout": BreakoutDevice, "pong": PongDevice}


class DeviceCollector:
    def __init__(self, model, env_num, num_simulations, device="cuda", max_episode_steps=200, episode_slots=8,
                 temperature=1.0, deterministic=False, noise_alpha=0.3, noise_weight=0.25, seed=0,
                 rng_mode="glibc", graph=True, poll_every=8, record_pred=False, support_scale=None,
                 categorical_distribution=True, env="cartpole", search_cfg=None):
        """search_cfg: the search's config keys (discount_factor, lstm_horizon_len, ...: the policy's)"""
        _lib.require_gpu()
        self.n, self.S = int(env_num), int(num_simulations)
        self.dev = torch.device(device)
        env_cls = DEVICE_ENVS[env] if isinstance(env, str) else env
        self.env = env_cls(self.n, self.dev)
        self.A = self.env.A
        self.T = int(max_episode_steps)
        self.E = int(episode_slots)
        self.temperature, self.deterministic = float(temperature), bool(deterministic)
        self.noise_alpha = float(noise_alpha)
        self.seed = int(seed) & 0xFFFFFFFF
        self.poll_every = int(poll_every)
        support_scale = self.env.support_scale if support_scale is None else int(support_scale)
        n, A, T, E, dev = self.n, self.A, self.T, self.E, self.dev
        self.rec_frames = torch.zeros((n, E, T + 1) + tuple(self.env.frame_shape), dtype=self.env.frame_dtype,
                                      device=dev)
        self.rec_action = torch.zeros((n, E, T), dtype=torch.int32, device=dev)
        self.rec_reward = torch.zeros((n, E, T), dtype=torch.float32, device=dev)
        self.rec_visits = torch.zeros((n, E, T, A), dtype=torch.int32, device=dev)
        self.rec_value = torch.zeros((n, E, T), dtype=torch.float32, device=dev)
        self.rec_pred = torch.zeros((n, E, T), dtype=torch.float32, device=dev) if record_pred else None
        self._pred_transform = None
        if record_pred:
            from .scaling_transform import InverseScalarTransform
            # the value head's own encoding (policy config model.categorical_distribution)
            self._pred_transform = InverseScalarTransform(support_scale, dev, bool(categorical_distribution))
        self._epoch = 0
        self.ep_len = torch.zeros((n, E), dtype=torch.int32, device=dev)
        self.ep_count = torch.zeros(n, dtype=torch.int32, device=dev)
        # each finished episode's return (the env's eval_episode_return: CartPole's reward sum, the Atari
        # game's unclipped score), carried in the packed block's row L (trajectory.py)
        self.ep_return = torch.zeros((n, E), dtype=torch.float32, device=dev)
        # device packing state (lzm_episodes_*): episodes returned per env, offsets, totals
        self._consumed_dev = torch.zeros(n, dtype=torch.int32, device=dev)
        self._ep_off = torch.zeros(n, dtype=torch.int32, device=dev)
        self._row_off = torch.zeros(n, dtype=torch.int64, device=dev)
        self._totals = torch.zeros(4, dtype=torch.int64, device=dev)
        me = weakref.ref(self)  # no collector <-> search-step reference cycle

        def epilogue(out):
            me()._env_step(out)

        sc = dict(search_cfg or {})
        self.search = DeviceSearchStep(model, n, self.S, [list(range(A))] * n, self.env.obs_shape, dev,
                                       noise_weight=noise_weight, seed=seed, rng_mode=rng_mode, graph=graph,
                                       epilogue=epilogue, support_scale=support_scale,
                                       discount_factor=sc.pop("discount_factor", 0.997), cfg_extra=sc)
        self.search.build_graph()
        self.reset()

    # backwards-compatible name of the recorded observations
    @property
    def rec_obs(self):
        return self.rec_frames

    def _env_step(self, out):
        pred = None
        if self._pred_transform is not None:  # predicted root value for priorities (muzero.py:667)
            pred = self._pred_transform(out["value_logits"]).reshape(-1)
        self.env.collect_step(self, out, pred)

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
        self.env.reset(self.search.obs, seed)
        g = torch.Generator(device=self.dev).manual_seed(seed)
        conc = torch.full((self.n, self.A), self.noise_alpha, dtype=torch.float64, device=self.dev)
        gam = torch._standard_gamma(conc, generator=g) if hasattr(torch, "_standard_gamma") else None
        noise = (gam / gam.sum(dim=1, keepdim=True)).float() if gam is not None else torch.full_like(conc, 0.5).float()
        self.search.noises.copy_(noise)
        self.ep_count.zero_()
        self.ep_len.zero_()
        self.ep_return.zero_()
        self._consumed_dev.zero_()
        self._consumed = np.zeros(self.n, dtype=np.int64)
        self._gathered_at = getattr(self, "envstep", 0)

    def step(self):
        """One env step for every env (one graph replay)."""
        self.search.step()
        self.envstep += self.n

    def _poll_until(self, n_episode):
        """step until n_episode new episodes have finished on this rank; returns the wall seconds"""
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
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
                return time.perf_counter() - t0

    def collect(self, n_episode, group=None, dst=None):
        """Step until `n_episode` new episodes have finished on this rank; returns (episodes, stats).

        Under an initialised torch.distributed process group (one collector per GPU, env-sharded)
        every rank's finished episodes are packed on its device and returned over the group
        (lightzero_amd.trajectory, RCCL over xGMI): to every rank (dst=None: all-gather) or to the
        learner rank `dst` alone (gather-to-learner; the other ranks get no episodes back), each tagged
        with its `rank`; the step / episode / duration statistics are sum-reduced on every rank
        (muzero_collector.py:709-712)."""
        steps0 = self.envstep
        el = self._poll_until(n_episode)
        blocks, stats = self._return_blocks(self.envstep - steps0, el, group, dst=dst)
        return self._unpack(blocks, stats)

    def collect_blocks(self, n_episode, group=None, to_host=False, dst=None):
        """collect() without the host unpacking: (the returned TrajBlocks in rank order, stats) — what a
        learner consumes directly (device tensors with to_host=False)."""
        steps0 = self.envstep
        el = self._poll_until(n_episode)
        return self._return_blocks(self.envstep - steps0, el, group, to_host, dst=dst)

    def gather_finished(self, group=None, dst=None):
        """The episodes finished since the last collect / gather, without stepping: packed on the
        device and returned over the process group as collect does. Returns (episodes, stats)."""
        blocks, stats = self.gather_blocks(group, to_host=True, dst=dst)
        return self._unpack(blocks, stats)

    def gather_blocks(self, group=None, to_host=False, dst=None):
        """gather_finished() without the host unpacking: (TrajBlocks in rank order, stats)."""
        steps = self.envstep - getattr(self, "_gathered_at", 0)
        return self._return_blocks(steps, 0.0, group, to_host, dst=dst)

    def _world(self, group):
        """the group's size when a process group is initialised (its collectives then carry the return, even
        with one rank), else 0"""
        return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 0

    def _check_search(self):
        """the fused searches' tie-break stream intact (lzm_check_errors raises) before their episodes leave"""
        roots = self.search.roots
        if roots is not None and roots.tree is not None:
            roots.tree.check_errors()

    def _return_blocks(self, steps, el, group, to_host=True, dst=None):
        self._check_search()
        block = self.pack_new()
        self._gathered_at = self.envstep
        world = self._world(group)
        coll = None
        if world >= 1:
            rank = dist.get_rank(group)
            torch.cuda.synchronize(self.dev)
            t0 = time.perf_counter()
            if dst is None:
                blocks = all_gather_packed(block, group, to_host=to_host)
            else:
                blocks = gather_packed(block, int(dst), group, to_host=to_host)
            tot_steps, tot_eps, tot_secs = allreduce_stats(steps, block.num_episodes, el, self.dev, group)
            torch.cuda.synchronize(self.dev)
            mine = wire_bytes(block)
            coll = dict(backend=str(dist.get_backend(group)), mode="all_gather" if dst is None else f"gather(dst={dst})",
                        ms=(time.perf_counter() - t0) * 1e3, bytes_sent=mine,
                        bytes_received=sum(wire_bytes(b) for r, b in enumerate(blocks) if r != rank))
        else:
            rank = 0
            world = 1
            blocks = [block.numpy() if to_host else block]
            tot_steps, tot_eps, tot_secs = steps, block.num_episodes, el
        stats = dict(envstep=steps, seconds=el, env_steps_per_s=steps / el if el else None,
                     sims_per_s=steps * self.S / el if el else None, rank=rank, world=world,
                     total_envstep=tot_steps, total_episodes=tot_eps, total_duration=tot_secs,
                     episodes=sum(b.num_episodes for b in blocks), rows=sum(b.rows for b in blocks),
                     payload_bytes=sum(b.nbytes for b in blocks), collective=coll)
        return blocks, stats

    def _unpack(self, blocks, stats):
        episodes = [e for r, b in enumerate(blocks) for e in unpack_episodes(b, self.A, r)]
        stats = dict(stats, episode_returns=[float(e["episode_return"]) for e in episodes])
        return episodes, stats

    def pack_new(self):
        """The episodes finished since the last pack, as one TrajBlock on the device (lzm_episodes_scan:
        offsets + totals, one 24-byte read-back to size the block; lzm_episodes_pack: the copy). Raises
        when a returned slot was overwritten (episode_slots too small for the poll interval)."""
        n, E = self.n, self.E
        call("lzm_episodes_scan", n, E, ptr(self.ep_count), ptr(self._consumed_dev), ptr(self.ep_len), ptr(self._ep_off),
             ptr(self._row_off), ptr(self._totals), stream_ptr())
        # one read-back: the totals and the counts they were taken at (the host mirror of `consumed`)
        snap = torch.cat([self._totals, self.ep_count.to(torch.int64)]).cpu().numpy()
        n_ep, rows, over = (int(v) for v in snap[:3])
        if over:
            raise RuntimeError("episode slots overwritten before collection: raise episode_slots or lower poll_every")
        has_pred = self.rec_pred is not None
        frames = torch.empty((rows,) + tuple(self.env.frame_shape), dtype=self.env.frame_dtype, device=self.dev)
        scalars = torch.empty((rows, scalar_width(self.A, has_pred)), dtype=torch.float32, device=self.dev)
        index = torch.empty((n_ep, 3), dtype=torch.int64, device=self.dev)
        fbytes = int(np.prod(self.env.frame_shape)) * self.rec_frames.element_size()
        if n_ep:
            call("lzm_episodes_pack", n, E, self.T, self.A, int(has_pred), fbytes, ptr(self.ep_count), ptr(self.ep_len),
                 ptr(self._consumed_dev), ptr(self._ep_off), ptr(self._row_off), ptr(self.rec_frames),
                 ptr(self.rec_action), ptr(self.rec_reward), ptr(self.rec_visits), ptr(self.rec_value),
                 ptr(self.rec_pred), ptr(self.ep_return), ptr(frames), ptr(scalars), ptr(index), stream_ptr())
        self._consumed = snap[4:].astype(np.int64)  # lzm_episodes_pack sets consumed = ep_count on the device
        return TrajBlock(frames, scalars, index, self.env.frame_scale)

    def pull_new(self):
        """The episodes finished since the last pull, on the host (one device pack + one copy):
        episode dicts in env order, each env's episodes in finishing order."""
        self._check_search()  # as collect() / gather_blocks()
        return unpack_episodes(self.pack_new(), self.A)
