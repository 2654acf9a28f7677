"""HBM-resident prioritized replay.

Layout on the GPU (all ``torch`` allocations on one device):

* ``frames``  u8 [F, 84*84]  -- every observed frame stored once (frame ring)
* ``s_ids`` / ``s2_ids`` int32 [C, 4] -- frame ids of the stacked s / s'
* ``action`` int32 [C], ``reward`` f32 [C] (n-step return), ``done`` f32 [C]
* the fanout-64 priority tree (``_apex_hip`` ``per_*`` kernels): fp32 leaves
  (sum + min), fp64 internal sums, fp32 internal mins
* ``max_prio`` f32 [1]; ``filled`` i64 [1] (slots written, read on device by the
  sampler so a captured graph sees the live fill level)

Frame dedup makes 1M transitions ~7.1 GB and 10M ~71 GB (fits 288 GB of HBM3E); the
reference's Python list of LazyFrames under one lock is replaced by device kernels
that never sync with the host.

API mirrors the reference buffer (``sample(B, beta)``, ``update_priorities``) but
everything stays on device: ``sample`` returns device tensors, priorities are
device tensors, nothing is copied to the host.
"""
from __future__ import annotations

import math

import torch

from .. import ops

FRAME_BYTES = 84 * 84


def tree_level_sizes(capacity: int) -> list[int]:
    sizes = [int(capacity)]
    while sizes[-1] > 1:
        sizes.append((sizes[-1] + 63) // 64)
    if len(sizes) == 1:  # capacity 1: still need one internal level
        sizes.append(1)
    return sizes


class HBMReplay:
    def __init__(self, capacity: int, n_envs: int, n_step: int = 3, alpha: float = 0.6,
                 device: str | torch.device = "cuda", frame_bytes: int = FRAME_BYTES,
                 frame_capacity: int | None = None, exact_mass: bool = True, seed: int = 0):
        self.hip = ops.hip()
        self.device = torch.device(device)
        self.capacity = int(capacity)
        self.n_envs = int(n_envs)
        self.alpha = float(alpha)
        self.frame_bytes = int(frame_bytes)
        # frames must outlive every transition that references them (see actor_kernels.hip)
        self.frame_capacity = int(frame_capacity or (self.capacity + (2 * n_step + 8) * self.n_envs))
        self.exact_mass = exact_mass
        self.seed = int(seed)
        dev = self.device
        C = self.capacity
        self.frames = torch.zeros(self.frame_capacity, self.frame_bytes, dtype=torch.uint8, device=dev)
        self.s_ids = torch.zeros(C, 4, dtype=torch.int32, device=dev)
        self.s2_ids = torch.zeros(C, 4, dtype=torch.int32, device=dev)
        self.action = torch.zeros(C, dtype=torch.int32, device=dev)
        self.reward = torch.zeros(C, dtype=torch.float32, device=dev)
        self.done = torch.zeros(C, dtype=torch.float32, device=dev)
        sizes = tree_level_sizes(C)
        self.level_sizes = sizes
        self.leaf_sum = torch.zeros(C, dtype=torch.float32, device=dev)
        self.leaf_min = torch.full((C,), math.inf, dtype=torch.float32, device=dev)
        self.node_sum = [torch.zeros(n, dtype=torch.float64, device=dev) for n in sizes[1:]]
        self.node_min = [torch.full((n,), math.inf, dtype=torch.float32, device=dev) for n in sizes[1:]]
        self.max_prio = torch.ones(1, dtype=torch.float32, device=dev)
        self.filled = torch.zeros(1, dtype=torch.int64, device=dev)
        self.sorted_scratch = torch.zeros(1024, dtype=torch.int32, device=dev)
        # batched-write scratch: per-slot dedup claims (all -1 between writes), the dirty
        # slot list, the last-block ticket of the level kernels
        self.owner = torch.full((C,), -1, dtype=torch.int32, device=dev)
        self.wlist = torch.zeros(2048, dtype=torch.int32, device=dev)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.tree = self.hip.make_tree(self.leaf_sum.data_ptr(), self.leaf_min.data_ptr(),
                                       [t.data_ptr() for t in self.node_sum], [t.data_ptr() for t in self.node_min],
                                       sizes)

    # ------------------------------------------------------------------ bytes
    def nbytes(self) -> int:
        tensors = [self.frames, self.s_ids, self.s2_ids, self.action, self.reward, self.done, self.leaf_sum,
                   self.leaf_min, *self.node_sum, *self.node_min]
        return sum(t.numel() * t.element_size() for t in tensors)

    def trans_ptrs(self) -> dict:
        return {"s_ids": self.s_ids.data_ptr(), "s2_ids": self.s2_ids.data_ptr(), "action": self.action.data_ptr(),
                "reward": self.reward.data_ptr(), "done": self.done.data_ptr()}

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    # ------------------------------------------------------------------ priorities
    def write_priorities(self, idx: torch.Tensor, prio: torch.Tensor | None, dedup: bool = True,
                         bumps: tuple = (), mix: tuple | None = None) -> None:
        """Set leaves for ``idx`` (int32) to prio**alpha (None = current max priority),
        then recompute all dirty ancestors level by level.  ``dedup`` resolves duplicate
        indices last-write-wins (B <= 1024); without it ``idx`` must be unique slots in
        ring order.  ``bumps``: up to two (int64 device counter, delta) pairs advanced by
        the same launch.  ``mix`` = (delta, lw, prio_out, loss_out): priorities derived
        in-kernel from TD errors, 0.9 max(delta) + 0.1 delta + 1e-6 (utils.py:77), and the
        loss mean of lw written to loss_out (dedup only)."""
        B = idx.numel()
        b = list(bumps) + [(None, 0)] * (2 - len(bumps))
        ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        self.hip.per_write_leaves(self.tree, idx.data_ptr(), 0 if prio is None else prio.data_ptr(), B, self.alpha,
                                  self.max_prio.data_ptr(), int(dedup), self.sorted_scratch.data_ptr(), ptr(b[0][0]),
                                  int(b[0][1]), ptr(b[1][0]), int(b[1][1]), self._stream(),
                                  *((0, 0, 0, 0) if mix is None else tuple(ptr(t) for t in mix)))

    def write_batch(self, pre: tuple | None = None, idx: torch.Tensor | None = None, prio: torch.Tensor | None = None,
                    mix: tuple | None = None, bump: torch.Tensor | None = None) -> None:
        """Fast batched tree update: ``pre`` = (slots int32 [E], raw priorities [E],
        counter advanced by E) -- an actor step's unique ring slots -- written first; then
        ``idx`` (int32 [B], duplicates last-write-wins) with ``prio`` or ``mix`` =
        (delta, lw, prio_out, loss_out) as in :meth:`write_priorities`; ``bump`` advanced
        by 1.  One leaves kernel + one wide kernel per big tree level."""
        ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        E = 0 if pre is None else pre[0].numel()
        B = 0 if idx is None else idx.numel()
        m = (None, None, None, None) if mix is None else mix
        self.hip.per_write_batch(self.tree, ptr(pre[0]) if pre else 0, ptr(pre[1]) if pre else 0, E,
                                 ptr(pre[2]) if pre else 0, ptr(idx), ptr(prio), B, ptr(m[0]), ptr(m[1]), ptr(m[2]),
                                 ptr(m[3]), ptr(bump), self.owner.data_ptr(), self.wlist.data_ptr(),
                                 self.max_prio.data_ptr(), self.alpha, self.ticket.data_ptr(), self._stream())

    update_priorities = write_priorities

    def sample_indices(self, B: int, out_idx: torch.Tensor, out_w: torch.Tensor, counter: torch.Tensor,
                       beta: float | torch.Tensor = 0.4, exclude_last: bool | None = None,
                       glob: torch.Tensor | None = None, shard: tuple | None = None, rows: tuple | None = None,
                       out_rows: dict | None = None, seed: int | None = None) -> None:
        """``glob`` (sharded replay): f32 [2] device tensor = (global min priority, this
        shard's IS-weight scale), see :mod:`apex_amd.parallel.sharded`; or ``shard`` =
        (exchanged fp32 slots [world, 2] = (mass, min priority) per shard, world, rank):
        the sampler derives both in-kernel.  ``rows`` = (staged table ptr dict, slot [E],
        prio [E]): an actor step's staged rows scattered into the tables by the same launch.
        ``out_rows`` (:meth:`row_buffers`): a private copy of every sampled row (frame ids,
        action, return, done) taken by the same launch -- the learner's sampled-ahead batch
        stays valid when the actor overwrites its slots before the batch is used."""
        excl = (not self.exact_mass) if exclude_last is None else exclude_last
        beta_ptr = beta.data_ptr() if isinstance(beta, torch.Tensor) else 0
        beta_c = 0.0 if isinstance(beta, torch.Tensor) else float(beta)
        sd = self.seed if seed is None else int(seed)
        self.hip.per_sample(self.tree, B, self.filled.data_ptr(), 0, beta_ptr, beta_c, sd, counter.data_ptr(),
                            out_idx.data_ptr(), out_w.data_ptr(), int(excl), self._stream(),
                            0 if glob is None else glob.data_ptr(),
                            *((0, 0, 0) if shard is None else (shard[0].data_ptr(), int(shard[1]), int(shard[2]))),
                            *((None, None, 0, 0, 0) if rows is None else
                              (rows[0], self.trans_ptrs(), rows[1].data_ptr(), rows[2].data_ptr(), rows[1].numel())),
                            *((None, None) if out_rows is None else
                              (self.trans_ptrs(), {k: t.data_ptr() for k, t in out_rows.items()})))

    def row_buffers(self, B: int) -> dict:
        """Private transition rows for ``B`` samples (``sample_indices(out_rows=)``), same
        dtypes and layout as the replay tables."""
        dev = self.device
        return {"s_ids": torch.zeros(B, 4, dtype=torch.int32, device=dev),
                "s2_ids": torch.zeros(B, 4, dtype=torch.int32, device=dev),
                "action": torch.zeros(B, dtype=torch.int32, device=dev),
                "reward": torch.zeros(B, dtype=torch.float32, device=dev),
                "done": torch.zeros(B, dtype=torch.float32, device=dev)}

    def pack_shard_slots(self, slots: torch.Tensor, world: int, rank: int) -> None:
        """slots[:] = 0 except slot ``rank`` = (root mass, root min priority) (fp32)."""
        assert slots.dtype == torch.float32 and slots.numel() >= 2 * world
        self.hip.pack_shard_slots(self.tree, slots.data_ptr(), world, rank, self._stream())

    def gather(self, idx: torch.Tensor, out_s, out_s2, out_a, out_r, out_d) -> None:
        self.hip.gather_transitions(self.frames.data_ptr(), self.frame_bytes, self.s_ids.data_ptr(),
                                    self.s2_ids.data_ptr(), self.action.data_ptr(), self.reward.data_ptr(),
                                    self.done.data_ptr(), idx.data_ptr(), idx.numel(), out_s.data_ptr(),
                                    out_s2.data_ptr(), out_a.data_ptr(), out_r.data_ptr(), out_d.data_ptr(),
                                    self._stream())

    def gather_frames(self, ids: torch.Tensor, out: torch.Tensor) -> None:
        N, stack = ids.shape
        self.hip.gather_frames(self.frames.data_ptr(), self.frame_bytes, ids.data_ptr(), N, stack, out.data_ptr(),
                               self._stream())

    # ------------------------------------------------------------------ convenience (allocating)
    def sample(self, batch_size: int, beta: float, counter: torch.Tensor | None = None):
        """Allocating convenience API: (s u8, a i64, r, s2 u8, d, w, idx) on device."""
        dev = self.device
        counter = counter if counter is not None else torch.zeros(1, dtype=torch.int64, device=dev)
        idx = torch.empty(batch_size, dtype=torch.int32, device=dev)
        w = torch.empty(batch_size, dtype=torch.float32, device=dev)
        self.sample_indices(batch_size, idx, w, counter, beta)
        s = torch.empty(batch_size, 4, 84, 84, dtype=torch.uint8, device=dev)
        s2 = torch.empty_like(s)
        a = torch.empty(batch_size, dtype=torch.int32, device=dev)  # gather_transitions_k writes int32
        r = torch.empty(batch_size, dtype=torch.float32, device=dev)
        d = torch.empty(batch_size, dtype=torch.float32, device=dev)
        self.gather(idx, s, s2, a, r, d)
        return s, a.long(), r, s2, d, w, idx

    def total_priority(self) -> float:
        return float(self.node_sum[-1][0].item())

    def min_priority(self) -> float:
        return float(self.node_min[-1][0].item())

    def __len__(self) -> int:
        return int(min(self.filled.item(), self.capacity))
