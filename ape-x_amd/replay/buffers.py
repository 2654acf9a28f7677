"""Host replay buffers with the reference API (memory.py:146-391).

* ``ReplayBuffer(size)``                         -- uniform ring (memory.py:146-205)
* ``PrioritizedReplayBuffer(size, alpha)``       -- PER, max-priority insert (208-320)
* ``CustomPrioritizedReplayBuffer(size, alpha)`` -- Ape-X: actor-computed priority on
  ``add``; observations (e.g. LazyFrames) are returned un-stacked (323-362)
* ``CustomPrioritizedReplayBuffer_AQL``          -- stores the candidate set ``a_mu``
  (364-391)

Transition payloads stay Python objects (like the reference) but every priority
operation is one native call into ``_apex_cpu.PERCore`` (no per-item Python tree
walk, no lock).  Sampling draws its B stratum offsets from Python's ``random`` in
the reference's order, so for equal seeds indices/weights match the reference
exactly.  ``exact_mass=False`` (default) reproduces the reference's exclusive-end
mass (the newest slot excluded); ``exact_mass=True`` samples over the
full mass.  The GPU/HBM replay used by the engine is :mod:`apex_amd.engine.hbm_replay`.
"""
from __future__ import annotations

import random

import numpy as np

from .. import ops
from .segment_tree import MinSegmentTree, SumSegmentTree


class ReplayBuffer:
    def __init__(self, size):
        self._storage = []
        self._maxsize = int(size)
        self._next_idx = 0

    def __len__(self):
        return len(self._storage)

    def _put(self, data):
        if self._next_idx >= len(self._storage):
            self._storage.append(data)
        else:
            self._storage[self._next_idx] = data
        self._next_idx = (self._next_idx + 1) % self._maxsize

    def add(self, obs_t, action, reward, obs_tp1, done):
        self._put((obs_t, action, reward, obs_tp1, done))

    def _encode_sample(self, idxes):
        cols = list(zip(*(self._storage[i] for i in idxes)))
        obs_t, act, rew, obs_tp1, done = cols
        return (np.array([np.asarray(o) for o in obs_t]), np.array([np.asarray(a) for a in act]), np.array(rew),
                np.array([np.asarray(o) for o in obs_tp1]), np.array(done))

    def sample(self, batch_size):
        idxes = [random.randint(0, len(self._storage) - 1) for _ in range(batch_size)]
        return self._encode_sample(idxes)


class PrioritizedReplayBuffer(ReplayBuffer):
    def __init__(self, size, alpha, exact_mass: bool = False):
        super().__init__(size)
        assert alpha >= 0
        self._alpha = alpha
        self._core = ops.cpu().PERCore(int(size), float(alpha))
        self._it_sum = SumSegmentTree._wrap(self._core.sum_tree())
        self._it_min = MinSegmentTree._wrap(self._core.min_tree())
        self._exact_mass = exact_mass

    @property
    def _max_priority(self):
        return self._core.max_priority

    @_max_priority.setter
    def _max_priority(self, v):
        self._core.max_priority = float(v)

    def add(self, *args, **kwargs):
        idx = self._next_idx
        super().add(*args, **kwargs)
        self._core.add_max(np.array([idx], dtype=np.int64))

    def _sample_proportional(self, batch_size):
        u = np.array([random.random() for _ in range(batch_size)], dtype=np.float64)
        return self._core.sample_proportional(u, len(self._storage), not self._exact_mass).tolist()

    def sample(self, batch_size, beta):
        assert beta > 0
        idxes = self._sample_proportional(batch_size)
        weights = self._core.weights(np.asarray(idxes, dtype=np.int64), len(self._storage), float(beta))
        encoded = self._encode_sample(idxes)
        return tuple(list(encoded) + [weights, idxes])

    def update_priorities(self, idxes, priorities):
        assert len(idxes) == len(priorities)
        self._core.update_priorities(np.asarray(idxes, dtype=np.int64),
                                     np.asarray(priorities, dtype=np.float64).reshape(-1), len(self._storage))


class CustomPrioritizedReplayBuffer(PrioritizedReplayBuffer):
    def add(self, state, action, reward, next_state, done, priority):
        idx = self._next_idx
        self._put((state, action, reward, next_state, done))
        self._core.add_with_priority(np.array([idx], dtype=np.int64), np.array([float(priority)]))

    def add_batch(self, states, actions, rewards, next_states, dones, priorities):
        """Insert a whole actor chunk with one native priority call."""
        n = len(priorities)
        idx = np.empty(n, dtype=np.int64)
        for i in range(n):
            idx[i] = self._next_idx
            self._put((states[i], actions[i], rewards[i], next_states[i], dones[i]))
        self._core.add_with_priority(idx, np.asarray(priorities, dtype=np.float64))

    def _encode_sample(self, idxes):
        obs_t, act, rew, obs_tp1, done = zip(*(self._storage[i] for i in idxes))
        return (list(obs_t), np.array([np.asarray(a) for a in act]), np.array([np.asarray(r) for r in rew]),
                list(obs_tp1), np.array([np.asarray(d) for d in done]))


class CustomPrioritizedReplayBuffer_AQL(PrioritizedReplayBuffer):
    def add(self, obs_t, action, reward, obs_tp1, done, a_mu):
        idx = self._next_idx
        self._storage_put_aql((obs_t, action, reward, obs_tp1, done, a_mu))
        self._core.add_max(np.array([idx], dtype=np.int64))

    def _storage_put_aql(self, data):
        if self._next_idx >= len(self._storage):
            self._storage.append(data)
        else:
            self._storage[self._next_idx] = data
        self._next_idx = int((self._next_idx + 1) % self._maxsize)

    def _encode_sample(self, idxes):
        obs_t, act, rew, obs_tp1, done, a_mu = zip(*(self._storage[i] for i in idxes))
        return (np.array([np.asarray(o) for o in obs_t]), np.array([np.asarray(a) for a in act]), np.array(rew),
                np.array([np.asarray(o) for o in obs_tp1]), np.array(done), np.array(a_mu))
