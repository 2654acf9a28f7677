"""Minimal gym-compatible spaces (gym is not installed in this image).

The reference branches on ``isinstance(env.action_space, gym.spaces.Box)`` and reads
``.n`` / ``.shape`` / ``.low`` / ``.high`` (model.py:175-186, 349-360); these classes
provide exactly that surface.  When a real ``gym`` is importable, ``is_box`` and
``is_discrete`` also accept its space classes.
"""
from __future__ import annotations

import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self.np_random = np.random.RandomState()

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def sample(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def contains(self, x):  # pragma: no cover - abstract
        raise NotImplementedError


class Discrete(Space):
    def __init__(self, n: int):
        super().__init__((), np.int64)
        self.n = int(n)

    def sample(self):
        return int(self.np_random.randint(self.n))

    def contains(self, x):
        try:
            x = int(x)
        except (TypeError, ValueError):
            return False
        return 0 <= x < self.n

    def __repr__(self):
        return f"Discrete({self.n})"

    def __eq__(self, other):
        return isinstance(other, Discrete) and other.n == self.n


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            low = np.asarray(low, dtype=dtype)
            high = np.asarray(high, dtype=dtype)
            shape = low.shape
        else:
            low = np.full(shape, low, dtype=dtype) if np.isscalar(low) else np.asarray(low, dtype=dtype)
            high = np.full(shape, high, dtype=dtype) if np.isscalar(high) else np.asarray(high, dtype=dtype)
        super().__init__(shape, dtype)
        self.low = low
        self.high = high

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return self.np_random.randint(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(self.dtype)
        lo = np.where(np.isfinite(self.low), self.low, -1e3)
        hi = np.where(np.isfinite(self.high), self.high, 1e3)
        return self.np_random.uniform(lo, hi, size=self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box{self.shape}"


def _gym_spaces():
    try:  # pragma: no cover - gym absent in this image
        import gym

        return gym.spaces
    except Exception:
        return None


def is_box(space) -> bool:
    if isinstance(space, Box):
        return True
    gs = _gym_spaces()
    return gs is not None and isinstance(space, gs.Box)


def is_discrete(space) -> bool:
    if isinstance(space, Discrete):
        return True
    gs = _gym_spaces()
    return gs is not None and isinstance(space, gs.Discrete)
