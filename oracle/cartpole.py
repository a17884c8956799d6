"""Test infrastructure: CartPole-v0 dynamics restated in numpy (float64), for checking the device
env of lightzero_amd/csrc/lzm_collect.h.

The reference env (zoo/classic_control/cartpole/envs/cartpole_lightzero_env.py:60-130) wraps
gymnasium.make('CartPole-v0'); gymnasium is not installed here, so this restates its published
classic-control CartPoleEnv.step (Euler, tau 0.02, force 10, gravity 9.8, cart 1.0, pole 0.1,
half-length 0.5, |x| > 2.4 or |theta| > 12 deg terminates, 200-step limit). Env parity is unpinned.
"""
import math

import numpy as np

GRAVITY, MASSCART, MASSPOLE, LENGTH, FORCE_MAG, TAU = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
TOTAL_MASS = MASSPOLE + MASSCART
POLEMASS_LENGTH = MASSPOLE * LENGTH
THETA_THRESHOLD = 12 * 2 * math.pi / 360
X_THRESHOLD = 2.4


def step(state, action):
    """state: float64 (4,) -> (new state, terminated)."""
    x, x_dot, theta, theta_dot = (float(v) for v in state)
    force = FORCE_MAG if action == 1 else -FORCE_MAG
    costheta, sintheta = math.cos(theta), math.sin(theta)
    temp = (force + POLEMASS_LENGTH * theta_dot * theta_dot * sintheta) / TOTAL_MASS
    thetaacc = (GRAVITY * sintheta - costheta * temp) / (LENGTH * (4.0 / 3.0 - MASSPOLE * costheta * costheta / TOTAL_MASS))
    xacc = temp - POLEMASS_LENGTH * thetaacc * costheta / TOTAL_MASS
    x = x + TAU * x_dot
    x_dot = x_dot + TAU * xacc
    theta = theta + TAU * theta_dot
    theta_dot = theta_dot + TAU * thetaacc
    term = x < -X_THRESHOLD or x > X_THRESHOLD or theta < -THETA_THRESHOLD or theta > THETA_THRESHOLD
    return np.array([x, x_dot, theta, theta_dot], dtype=np.float64), bool(term)
