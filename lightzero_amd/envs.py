"""Env managers for the collector: a host CartPole-v0 behind DI-engine's BaseEnvManager surface, and
the marker for the device-resident CartPole of the fast collector path.

The reference collects through DI-engine env managers (`SubprocessEnvManager`,
cartpole_muzero_config.py:70) over `CartPoleEnv` (zoo/classic_control/cartpole/envs/
cartpole_lightzero_env.py:14-130, which wraps gymnasium.make('CartPole-v0')). Neither DI-engine nor
gymnasium is installed here, so:

- `CartPoleEnv` restates gymnasium's classic-control CartPole (float64 state, Euler, tau 0.02,
  |x| > 2.4 or |theta| > 12 deg terminates, 200-step TimeLimit, reset U(-0.05, 0.05)^4 from a
  per-env numpy Generator) with LightZero's dict observations
  {'observation' float32 [4], 'action_mask' int8 [2], 'to_play' -1} and
  info['eval_episode_return'] at the end. Env parity is unpinned (gymnasium absent). Each env owns
  its Generator, so env resets never consume the global numpy stream the policy draws from (the
  reference's envs live in subprocesses with their own streams).
- `SyncEnvManager` is the BaseEnvManager surface MuZeroCollector uses (env_num, ready_obs,
  step(actions) -> {env_id: timestep}, reset, launch, close, action_space), stepping in-process
  and auto-resetting finished envs as DI-engine's managers do.
- `DeviceCartPoleEnvManager` / `DeviceBreakoutEnvManager` select MuZeroCollector's device path: the
  env state lives in HBM and steps inside the collect graph (lzm_collect.h, lzm_atari.h); these
  objects only carry the env kind, shape and seed.
"""
import math
from collections import namedtuple

import numpy as np

BaseEnvTimestep = namedtuple("BaseEnvTimestep", ["obs", "reward", "done", "info"])


class Discrete:
    """the slice of gymnasium.spaces.Discrete the collector and GameSegment read"""

    def __init__(self, n):
        self.n = int(n)

    def __repr__(self):
        return f"Discrete({self.n})"


class CartPoleEnv:
    GRAVITY, MASSCART, MASSPOLE, LENGTH, FORCE_MAG, TAU = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    THETA_THRESHOLD = 12 * 2 * math.pi / 360
    X_THRESHOLD = 2.4
    MAX_EPISODE_STEPS = 200  # CartPole-v0's TimeLimit

    def __init__(self, seed=0):
        self.action_space = Discrete(2)
        self._rng = np.random.default_rng(seed)
        self._state = None
        self._t = 0
        self._return = 0.0

    def _obs(self):
        return {"observation": np.array(self._state, dtype=np.float32), "action_mask": np.ones(2, "int8"),
                "to_play": -1}

    def reset(self):
        self._state = self._rng.uniform(low=-0.05, high=0.05, size=(4,))
        self._t = 0
        self._return = 0.0
        return self._obs()

    def step(self, action):
        if isinstance(action, np.ndarray) and action.shape == (1,):
            action = action.squeeze()
        x, x_dot, theta, theta_dot = (float(v) for v in self._state)
        force = self.FORCE_MAG if int(action) == 1 else -self.FORCE_MAG
        costheta, sintheta = math.cos(theta), math.sin(theta)
        total_mass = self.MASSPOLE + self.MASSCART
        pml = self.MASSPOLE * self.LENGTH
        temp = (force + pml * theta_dot * theta_dot * sintheta) / total_mass
        thetaacc = (self.GRAVITY * sintheta - costheta * temp) / (
            self.LENGTH * (4.0 / 3.0 - self.MASSPOLE * costheta * costheta / total_mass))
        xacc = temp - pml * thetaacc * costheta / total_mass
        x = x + self.TAU * x_dot
        x_dot = x_dot + self.TAU * xacc
        theta = theta + self.TAU * theta_dot
        theta_dot = theta_dot + self.TAU * thetaacc
        self._state = np.array([x, x_dot, theta, theta_dot], dtype=np.float64)
        self._t += 1
        terminated = x < -self.X_THRESHOLD or x > self.X_THRESHOLD or theta < -self.THETA_THRESHOLD or \
            theta > self.THETA_THRESHOLD
        done = bool(terminated) or self._t >= self.MAX_EPISODE_STEPS
        rew = 1.0
        self._return += rew
        info = {"eval_episode_return": self._return} if done else {}
        return BaseEnvTimestep(self._obs(), rew, done, info)

    def close(self):
        pass


class SyncEnvManager:
    """In-process BaseEnvManager surface over a list of envs (DI-engine's env managers are absent)."""

    def __init__(self, envs):
        self._envs = list(envs)
        self.env_num = len(self._envs)
        self.action_space = self._envs[0].action_space
        self._ready = {}
        self._env_states = {}
        self._closed = False
        self._launched = False

    @classmethod
    def cartpole(cls, env_num, seed=0):
        return cls([CartPoleEnv(seed + i) for i in range(env_num)])

    def launch(self):
        """reset every env once (idempotent, like DI-engine's launch of a running manager)"""
        if self._launched:
            return
        self._launched = True
        self._ready = {i: e.reset() for i, e in enumerate(self._envs)}
        self._env_states = {i: "run" for i in range(self.env_num)}

    @property
    def ready_obs(self):
        self.launch()
        return dict(self._ready)

    def step(self, actions):
        out = {}
        for env_id in sorted(actions):
            ts = self._envs[env_id].step(actions[env_id])
            out[env_id] = ts
            self._ready[env_id] = self._envs[env_id].reset() if ts.done else ts.obs
        return out

    def reset(self, reset_param=None):
        ids = range(self.env_num) if reset_param is None else list(reset_param)
        for i in ids:
            self._ready[i] = self._envs[i].reset()

    def close(self):
        if not self._closed:
            for e in self._envs:
                e.close()
            self._closed = True


class DeviceEnvManager:
    """env_num envs resident on the GPU (lightzero_amd.collector.DEVICE_ENVS): handing one to
    MuZeroCollector selects its device path. seed keys the envs' Philox reset streams."""
    env_kind = None
    actions = None
    observation_shape = None
    frame_stack = 1

    def __init__(self, env_num, seed=0, max_episode_steps=200):
        self.env_num = int(env_num)
        self.seed = int(seed)
        self.max_episode_steps = int(max_episode_steps)
        self.action_space = Discrete(self.actions)

    def launch(self):
        pass

    def reset(self, reset_param=None):
        pass

    def close(self):
        pass


class DeviceCartPoleEnvManager(DeviceEnvManager):
    """CartPole-v0 (config 2) on the device (lzm_cartpole_* kernels)."""
    env_kind = "cartpole"
    actions = 2
    observation_shape = (4,)
    frame_stack = 1


class DeviceBreakoutEnvManager(DeviceEnvManager):
    """The Atari image env of config 5 on the device (lzm_atari_* kernels): Breakout's action set and
    frame format — 4 x 64 x 64 stacked grey frames, one recorded per step — as a stand-in game (ALE
    is not installed)."""
    env_kind = "breakout"
    actions = 4
    observation_shape = (4, 64, 64)
    frame_stack = 4

    def __init__(self, env_num, seed=0, max_episode_steps=400):
        super().__init__(env_num, seed, max_episode_steps)


class DevicePongEnvManager(DeviceBreakoutEnvManager):
    """The Atari image env of config 3 (Pong EfficientZero) on the device (lzm_pong_* kernels): Pong's action set
    {NOOP, FIRE, RIGHT, LEFT, RIGHTFIRE, LEFTFIRE} and frame format — 4 x 64 x 64 stacked grey frames, one
    recorded per step — as a stand-in game (ALE is not installed)."""
    env_kind = "pong"
    actions = 6
