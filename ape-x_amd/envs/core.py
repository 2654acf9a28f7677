"""gym-0.12-style ``Env`` / ``Wrapper`` base classes and the env registry.

The reference talks to environments only through ``gym.make(id)``, ``reset()``,
``step(a) -> (obs, r, done, info)``, ``seed``, ``render``, ``close``,
``env.unwrapped.spec.id`` and the Atari extras ``get_action_meanings()`` /
``ale.lives()`` / ``np_random`` (origin_repo/wrapper.py:11-124, ApeX.py:19-42).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np


@dataclass
class EnvSpec:
    id: str
    max_episode_steps: int | None = None


class Env:
    observation_space = None
    action_space = None
    reward_range = (-float("inf"), float("inf"))
    metadata = {"render.modes": ["rgb_array"]}
    spec: EnvSpec | None = None

    def __init__(self):
        self.np_random = np.random.RandomState()

    @property
    def unwrapped(self):
        return self

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        if self.action_space is not None:
            self.action_space.seed(seed)
        return [seed]

    def reset(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def step(self, action):  # pragma: no cover - abstract
        raise NotImplementedError

    def render(self, mode="rgb_array"):
        return None

    def close(self):
        pass


class Wrapper(Env):
    def __init__(self, env):
        self.env = env
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self.reward_range = env.reward_range
        self.spec = getattr(env, "spec", None)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def seed(self, seed=None):
        return self.env.seed(seed)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, action):
        return self.env.step(action)

    def render(self, mode="rgb_array"):
        return self.env.render(mode)

    def close(self):
        return self.env.close()


class ObservationWrapper(Wrapper):
    def reset(self, **kwargs):
        return self.observation(self.env.reset(**kwargs))

    def step(self, action):
        obs, r, d, info = self.env.step(action)
        return self.observation(obs), r, d, info

    def observation(self, obs):  # pragma: no cover - abstract
        raise NotImplementedError


class RewardWrapper(Wrapper):
    def step(self, action):
        obs, r, d, info = self.env.step(action)
        return obs, self.reward(r), d, info

    def reward(self, r):  # pragma: no cover - abstract
        raise NotImplementedError


class TimeLimit(Wrapper):
    """origin_repo/wrapper.py:282-298."""

    def __init__(self, env, max_episode_steps=None):
        super().__init__(env)
        self._max_episode_steps = max_episode_steps
        self._elapsed_steps = 0

    def step(self, ac):
        observation, reward, done, info = self.env.step(ac)
        self._elapsed_steps += 1
        if self._max_episode_steps is not None and self._elapsed_steps >= self._max_episode_steps:
            done = True
            info["TimeLimit.truncated"] = True
        return observation, reward, done, info

    def reset(self, **kwargs):
        self._elapsed_steps = 0
        return self.env.reset(**kwargs)


_REGISTRY: dict[str, tuple[Callable[[], Env], int | None]] = {}


def register(env_id: str, entry: Callable[[], Env], max_episode_steps: int | None = None) -> None:
    _REGISTRY[env_id] = (entry, max_episode_steps)


def registered() -> list[str]:
    from . import classic, atari  # noqa: F401  (populate registry)

    return sorted(_REGISTRY)


def make(env_id: str) -> Env:
    """``gym.make`` equivalent.  Atari ids (``*NoFrameskip-v4`` etc.) resolve to the
    seeded synthetic Atari emulator in :mod:`apex_amd.envs.atari` (ALE is not
    available here); a real ``gym`` is used only if installed and ``APEX_USE_GYM=1``."""
    import os

    from . import classic, atari  # noqa: F401

    if os.environ.get("APEX_USE_GYM") == "1":  # pragma: no cover - gym absent here
        import gym

        return gym.make(env_id)
    if env_id not in _REGISTRY:
        if atari.is_atari_id(env_id):
            atari.register_atari(env_id)
        else:
            raise KeyError(f"unknown env id {env_id!r}; known: {sorted(_REGISTRY)}")
    entry, max_steps = _REGISTRY[env_id]
    env = entry()
    env.spec = EnvSpec(env_id, max_steps)
    env.unwrapped.spec = env.spec
    if max_steps is not None:
        env = TimeLimit(env, max_steps)
        env.spec = EnvSpec(env_id, max_steps)
    return env
