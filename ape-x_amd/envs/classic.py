"""Classic-control environments used by the reference's top-level trainers.

* CartPole-v0 / -v1   -- DQN.py:126, AQL_dis.py:145 (BASELINE config 1)
* MountainCar-v0      -- ApeX.py:92
* Pendulum-v0         -- AQL.py:160 (continuous action)
* MountainCarContinuous-v0
* BipedalWalker-v3    -- AQL_dis.py:145 comment / BASELINE config 4.  Box2D is not
  available, so this is a *shape-faithful stand-in*: 24-d observation, 4-d action in
  [-1, 1], 1600-step limit, -100 on "falling", with smooth synthetic dynamics.  It is
  a throughput/plumbing workload, not the physics benchmark.

Dynamics of CartPole / MountainCar / Pendulum follow the published equations of the
classic-control suite (Barto et al. 1983; Moore 1990).
"""
from __future__ import annotations

import math

import numpy as np

from .core import Env, register
from .spaces import Box, Discrete


class CartPoleEnv(Env):
    def __init__(self):
        super().__init__()
        self.gravity, self.masscart, self.masspole = 9.8, 1.0, 0.1
        self.total_mass = self.masspole + self.masscart
        self.length = 0.5
        self.polemass_length = self.masspole * self.length
        self.force_mag, self.tau = 10.0, 0.02
        self.theta_threshold_radians = 12 * 2 * math.pi / 360
        self.x_threshold = 2.4
        high = np.array([self.x_threshold * 2, np.finfo(np.float32).max,
                         self.theta_threshold_radians * 2, np.finfo(np.float32).max], dtype=np.float32)
        self.action_space = Discrete(2)
        self.observation_space = Box(-high, high, dtype=np.float32)
        self.state = None
        self.steps_beyond_done = None

    def step(self, action):
        action = int(action)
        assert self.action_space.contains(action), f"{action!r} invalid"
        x, x_dot, theta, theta_dot = self.state
        force = self.force_mag if action == 1 else -self.force_mag
        costheta, sintheta = math.cos(theta), math.sin(theta)
        temp = (force + self.polemass_length * theta_dot * theta_dot * sintheta) / self.total_mass
        thetaacc = (self.gravity * sintheta - costheta * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * costheta * costheta / self.total_mass))
        xacc = temp - self.polemass_length * thetaacc * costheta / self.total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * xacc
        theta = theta + self.tau * theta_dot
        theta_dot = theta_dot + self.tau * thetaacc
        self.state = (x, x_dot, theta, theta_dot)
        done = bool(x < -self.x_threshold or x > self.x_threshold
                    or theta < -self.theta_threshold_radians or theta > self.theta_threshold_radians)
        if not done:
            reward = 1.0
        elif self.steps_beyond_done is None:
            self.steps_beyond_done = 0
            reward = 1.0
        else:
            self.steps_beyond_done += 1
            reward = 0.0
        return np.array(self.state, dtype=np.float32), reward, done, {}

    def reset(self):
        self.state = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
        self.steps_beyond_done = None
        return np.array(self.state, dtype=np.float32)


class MountainCarEnv(Env):
    def __init__(self):
        super().__init__()
        self.min_position, self.max_position = -1.2, 0.6
        self.max_speed, self.goal_position = 0.07, 0.5
        self.force, self.gravity = 0.001, 0.0025
        low = np.array([self.min_position, -self.max_speed], dtype=np.float32)
        high = np.array([self.max_position, self.max_speed], dtype=np.float32)
        self.action_space = Discrete(3)
        self.observation_space = Box(low, high, dtype=np.float32)
        self.state = None

    def step(self, action):
        position, velocity = self.state
        velocity += (int(action) - 1) * self.force + math.cos(3 * position) * (-self.gravity)
        velocity = float(np.clip(velocity, -self.max_speed, self.max_speed))
        position += velocity
        position = float(np.clip(position, self.min_position, self.max_position))
        if position == self.min_position and velocity < 0:
            velocity = 0.0
        done = bool(position >= self.goal_position)
        self.state = (position, velocity)
        return np.array(self.state, dtype=np.float32), -1.0, done, {}

    def reset(self):
        self.state = (float(self.np_random.uniform(low=-0.6, high=-0.4)), 0.0)
        return np.array(self.state, dtype=np.float32)


class MountainCarContinuousEnv(MountainCarEnv):
    def __init__(self):
        super().__init__()
        self.power = 0.0015
        self.action_space = Box(-1.0, 1.0, shape=(1,), dtype=np.float32)

    def step(self, action):
        position, velocity = self.state
        force = min(max(float(np.asarray(action).reshape(-1)[0]), -1.0), 1.0)
        velocity += force * self.power - 0.0025 * math.cos(3 * position)
        velocity = min(max(velocity, -self.max_speed), self.max_speed)
        position = min(max(position + velocity, self.min_position), self.max_position)
        if position == self.min_position and velocity < 0:
            velocity = 0.0
        done = bool(position >= self.goal_position)
        reward = (100.0 if done else 0.0) - 0.1 * force ** 2
        self.state = (position, velocity)
        return np.array(self.state, dtype=np.float32), reward, done, {}


class PendulumEnv(Env):
    def __init__(self):
        super().__init__()
        self.max_speed, self.max_torque, self.dt = 8.0, 2.0, 0.05
        self.g, self.m, self.l = 10.0, 1.0, 1.0
        high = np.array([1.0, 1.0, self.max_speed], dtype=np.float32)
        self.action_space = Box(-self.max_torque, self.max_torque, shape=(1,), dtype=np.float32)
        self.observation_space = Box(-high, high, dtype=np.float32)
        self.state = None

    @staticmethod
    def _angle_normalize(x):
        return ((x + np.pi) % (2 * np.pi)) - np.pi

    def step(self, u):
        th, thdot = self.state
        u = float(np.clip(np.asarray(u, dtype=np.float64).reshape(-1)[0], -self.max_torque, self.max_torque))
        costs = self._angle_normalize(th) ** 2 + 0.1 * thdot ** 2 + 0.001 * (u ** 2)
        newthdot = thdot + (-3 * self.g / (2 * self.l) * np.sin(th + np.pi) + 3.0 / (self.m * self.l ** 2) * u) * self.dt
        newth = th + newthdot * self.dt
        newthdot = float(np.clip(newthdot, -self.max_speed, self.max_speed))
        self.state = np.array([newth, newthdot])
        return self._obs(), -float(costs), False, {}

    def reset(self):
        high = np.array([np.pi, 1.0])
        self.state = self.np_random.uniform(low=-high, high=high)
        return self._obs()

    def _obs(self):
        th, thdot = self.state
        return np.array([np.cos(th), np.sin(th), thdot], dtype=np.float32)


class BipedalWalkerShapedEnv(Env):
    """24-d obs / 4-d action stand-in for BipedalWalker-v3 (see module docstring)."""

    def __init__(self):
        super().__init__()
        self.action_space = Box(-1.0, 1.0, shape=(4,), dtype=np.float32)
        high = np.full(24, np.inf, dtype=np.float32)
        self.observation_space = Box(-high, high, dtype=np.float32)
        rng = np.random.RandomState(1234)  # fixed "terrain" dynamics, independent of the seed
        self._A = (np.eye(24) * 0.95 + rng.normal(0, 0.02, (24, 24))).astype(np.float64)
        self._B = rng.normal(0, 0.3, (24, 4)).astype(np.float64)
        self._w = rng.normal(0, 1.0, 24)
        self.state = None
        self.hull_x = 0.0

    def reset(self):
        self.state = self.np_random.normal(0, 0.1, 24)
        self.hull_x = 0.0
        return self.state.astype(np.float32)

    def step(self, action):
        a = np.clip(np.asarray(action, dtype=np.float64).reshape(4), -1.0, 1.0)
        self.state = self._A @ self.state + self._B @ a + self.np_random.normal(0, 0.01, 24)
        self.state = np.tanh(self.state)
        progress = float(self._w @ self.state) * 0.05
        self.hull_x += progress
        reward = progress - 0.00035 * 80.0 * float(np.abs(a).sum())
        done = False
        if abs(self.state[0]) > 0.995:  # "hull touches ground"
            reward, done = -100.0, True
        return self.state.astype(np.float32), reward, done, {}


register("CartPole-v0", CartPoleEnv, 200)
register("CartPole-v1", CartPoleEnv, 500)
register("MountainCar-v0", MountainCarEnv, 200)
register("MountainCarContinuous-v0", MountainCarContinuousEnv, 999)
register("Pendulum-v0", PendulumEnv, 200)
register("Pendulum-v1", PendulumEnv, 200)
register("BipedalWalker-v3", BipedalWalkerShapedEnv, 1600)
