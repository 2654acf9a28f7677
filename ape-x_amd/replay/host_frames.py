"""Host-memory prioritized replay for the replay *role* (origin_repo/replay.py:19-146;
SURVEY R2, §5.7).

The reference replay server keeps a Python list of LazyFrames tuples behind one
asyncio lock.  This server-side store keeps:

* **frame mode** (image observations): a u8 frame ring ``[F, frame_bytes]`` where
  each frame pushed by an actor is stored **once**; transitions hold the ring slots
  of their 4-frame s / s' stacks (the host twin of the HBM frame ring in
  :mod:`apex_amd.engine.hbm_replay`).  Actors send frame ids (per-actor sequence
  numbers) plus only the frames the replay has not seen yet.
* **vector mode**: ``[C, obs_dim]`` float arrays.

Priorities live in the native ``_apex_cpu.PERCore`` (sum/min trees, stratified
proportional sampling, IS weights); ``exact_mass=False`` keeps the reference's
exclusive-end mass.  Sampling uses a seeded generator (the reference
seeds from the wall clock, Q12).
"""
from __future__ import annotations

import numpy as np

from .. import ops


class HostReplay:
    def __init__(self, capacity: int, alpha: float = 0.6, frame_mode: bool = True, obs_shape=(4, 84, 84),
                 n_actors: int = 1, send_interval: int = 50, exact_mass: bool = False, seed: int = 0,
                 seq_window: int = 4096):
        self.capacity = int(capacity)
        self.frame_mode = frame_mode
        self.obs_shape = tuple(obs_shape)
        self.exact_mass = exact_mass
        self.core = ops.cpu().PERCore(self.capacity, float(alpha))
        self.rng = np.random.default_rng(seed)
        C = self.capacity
        self.action = np.zeros(C, dtype=np.int64)
        self.reward = np.zeros(C, dtype=np.float32)
        self.done = np.zeros(C, dtype=np.float32)
        if frame_mode:
            self.stack = self.obs_shape[0]
            self.frame_shape = self.obs_shape[1:]
            self.frame_bytes = int(np.prod(self.frame_shape))
            # frames are evicted FIFO; slack keeps every frame a live transition references
            self.frame_capacity = C + int(n_actors) * 4 * (send_interval + 16) + 1024
            self.frames = np.zeros((self.frame_capacity, self.frame_bytes), dtype=np.uint8)
            self.s_slot = np.zeros((C, self.stack), dtype=np.int64)
            self.s2_slot = np.zeros((C, self.stack), dtype=np.int64)
            self.frame_ptr = 0
            self.seq_window = int(seq_window)
            self.slot_of: dict[int, np.ndarray] = {}
        else:
            self.s = np.zeros((C, *self.obs_shape), dtype=np.float32)
            self.s2 = np.zeros((C, *self.obs_shape), dtype=np.float32)
        self.next_idx = 0
        self.size = 0
        self.pushed = 0

    def __len__(self) -> int:
        return self.size

    # ------------------------------------------------------------------ insert
    def _store_frames(self, actor: int, seqs: np.ndarray, frames: np.ndarray) -> None:
        tbl = self.slot_of.get(actor)
        if tbl is None:
            tbl = self.slot_of[actor] = np.full(self.seq_window, -1, dtype=np.int64)
        k = len(seqs)
        if k == 0:
            return
        slots = (self.frame_ptr + np.arange(k)) % self.frame_capacity
        self.frames[slots] = frames.reshape(k, self.frame_bytes)
        tbl[seqs % self.seq_window] = slots
        self.frame_ptr = int((self.frame_ptr + k) % self.frame_capacity)

    def _slots(self, actor: int, seqs: np.ndarray) -> np.ndarray:
        tbl = self.slot_of[actor]
        out = tbl[seqs % self.seq_window]
        if (out < 0).any():
            raise ValueError(f"actor {actor} referenced a frame it never sent")
        return out

    def add_chunk(self, actor: int, msg: dict) -> int:
        """Insert one actor chunk (see :class:`apex_amd.roles.common.ChunkEncoder`)."""
        n = len(msg["prio"])
        if n == 0:
            return 0
        idx = (self.next_idx + np.arange(n)) % self.capacity
        if self.frame_mode:
            self._store_frames(actor, msg["seq"], msg["frames"])
            self.s_slot[idx] = self._slots(actor, msg["s"])
            self.s2_slot[idx] = self._slots(actor, msg["s2"])
        else:
            self.s[idx] = msg["s"].reshape(n, *self.obs_shape)
            self.s2[idx] = msg["s2"].reshape(n, *self.obs_shape)
        self.action[idx] = msg["a"]
        self.reward[idx] = msg["r"]
        self.done[idx] = msg["d"]
        self.core.add_with_priority(idx.astype(np.int64), msg["prio"].astype(np.float64))
        self.next_idx = int((self.next_idx + n) % self.capacity)
        self.size = min(self.capacity, self.size + n)
        self.pushed += n
        return n

    # ------------------------------------------------------------------ sample / update
    def sample(self, batch_size: int, beta: float) -> dict:
        u = self.rng.random(batch_size)
        idx = np.asarray(self.core.sample_proportional(u, self.size, not self.exact_mass), dtype=np.int64)
        w = np.asarray(self.core.weights(idx, self.size, float(beta)), dtype=np.float32)
        if self.frame_mode:
            s = self.frames[self.s_slot[idx]].reshape(batch_size, self.stack, *self.frame_shape)
            s2 = self.frames[self.s2_slot[idx]].reshape(batch_size, self.stack, *self.frame_shape)
        else:
            s, s2 = self.s[idx], self.s2[idx]
        return {"s": s, "a": self.action[idx], "r": self.reward[idx], "s2": s2, "d": self.done[idx], "w": w,
                "idx": idx}

    def update_priorities(self, idx: np.ndarray, prios: np.ndarray) -> None:
        self.core.update_priorities(np.asarray(idx, dtype=np.int64), np.asarray(prios, dtype=np.float64).reshape(-1),
                                    self.size)

    def nbytes(self) -> int:
        arrs = [self.action, self.reward, self.done]
        arrs += [self.frames, self.s_slot, self.s2_slot] if self.frame_mode else [self.s, self.s2]
        return int(sum(a.nbytes for a in arrs))
