"""Actor -> replay experience push for the central-replay topology.

Central topology: rank 0 owns the single HBM replay and the learner; ranks 1..W-1 run
GPU actor shards only.  Each remote rank's actor writes into a *local mirror* of its
region of the rank-0 replay (same frame-ring and transition-slot geometry), so one
actor step produces, at positions the shard itself reports:

* E new frames (one per env, local frame slots in ``ActorShard.new_frame``), and
* E transition rows (local slots in ``ActorShard.slot``; priority 0 = no row emitted).

Per actor step the remote rank gathers them on device (inside its captured actor graph)
and sends one frame tensor ``[E, frame_bytes]`` u8 and one metadata tensor ``[E, 14]``
int32 -- point-to-point over RCCL/xGMI with the ``nccl`` backend (a 1.8 MB message per
256-env step), or staged through host memory with ``gloo``.  Rank 0 scatters them into
region r (frame ids re-based by the region's frame offset) and writes the priorities
into the tree.  Reference equivalent: actor pickles 50
transitions and pushes them over ZeroMQ to the replay process (actor.py:105-115,
replay.py:77-107).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

META_COLS = 14


def pack_meta(s_ids, s2_ids, action, reward, done, prio, slot, fslot, out: torch.Tensor | None = None):
    """[E, 14] int32 packing of one actor step (floats as raw bits): s_ids 4 | s2_ids 4 |
    action | reward | done | priority | local transition slot | local new-frame slot.
    Pure device ops (graph-capturable)."""
    E = action.numel()
    out = out if out is not None else torch.empty(E, META_COLS, dtype=torch.int32, device=action.device)
    out[:, 0:4].copy_(s_ids.reshape(E, 4))
    out[:, 4:8].copy_(s2_ids.reshape(E, 4))
    out[:, 8].copy_(action.reshape(E))
    out[:, 9].copy_(reward.reshape(E).contiguous().view(torch.int32))
    out[:, 10].copy_(done.reshape(E).contiguous().view(torch.int32))
    out[:, 11].copy_(prio.reshape(E).contiguous().view(torch.int32))
    out[:, 12].copy_(slot.reshape(E))
    out[:, 13].copy_(fslot.reshape(E))
    return out


class Region:
    """Where remote rank r's experience lives inside the rank-0 replay."""

    def __init__(self, slot_base: int, n_slots: int, frame_base: int, n_frames: int):
        self.slot_base, self.n_slots = int(slot_base), int(n_slots)
        self.frame_base, self.n_frames = int(frame_base), int(n_frames)


def apply_packet(tables: dict, region: Region, frames: torch.Tensor, meta: torch.Tensor):
    """Write one remote actor step into region ``region`` of the rank-0 tables; returns
    (global slots int32 [E], priorities f32 [E]) for the priority-tree write."""
    fslot = meta[:, 13].long() + region.frame_base
    tables["frames"].index_copy_(0, fslot, frames)
    slot = meta[:, 12].long() + region.slot_base
    ids = meta[:, 0:8] + region.frame_base
    tables["s_ids"].index_copy_(0, slot, ids[:, 0:4].contiguous())
    tables["s2_ids"].index_copy_(0, slot, ids[:, 4:8].contiguous())
    tables["action"].index_copy_(0, slot, meta[:, 8].contiguous())
    tables["reward"].index_copy_(0, slot, meta[:, 9].contiguous().view(torch.float32))
    tables["done"].index_copy_(0, slot, meta[:, 10].contiguous().view(torch.float32))
    return slot.to(torch.int32), meta[:, 11].contiguous().view(torch.float32)


class _P2P:
    def __init__(self, device: torch.device, group=None):
        self.group = group
        backend = dist.get_backend(group)
        self.via_host = device.type == "cuda" and backend != "nccl"  # gloo: stage through host memory
        self.works: list = []

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []


class ExperienceSender(_P2P):
    def __init__(self, E: int, frame_bytes: int, device, dst: int = 0, group=None):
        super().__init__(torch.device(device), group)
        self.dst = dst
        self.meta = torch.empty(E, META_COLS, dtype=torch.int32, device=device)
        if self.via_host:
            self.h_frames = torch.empty(E, frame_bytes, dtype=torch.uint8).pin_memory() \
                if torch.cuda.is_available() else torch.empty(E, frame_bytes, dtype=torch.uint8)
            self.h_meta = torch.empty(E, META_COLS, dtype=torch.int32)

    def send(self, frames: torch.Tensor, meta: torch.Tensor) -> None:
        self.wait()  # one packet in flight: the staging buffers are reused
        if self.via_host:
            self.h_frames.copy_(frames)
            self.h_meta.copy_(meta)
            frames, meta = self.h_frames, self.h_meta
        self.works = [dist.isend(frames.contiguous(), self.dst, group=self.group),
                      dist.isend(meta.contiguous(), self.dst, group=self.group)]


class ExperienceReceiver(_P2P):
    def __init__(self, E: int, frame_bytes: int, device, sources, group=None):
        super().__init__(torch.device(device), group)
        self.sources = list(sources)
        dev = device if not self.via_host else "cpu"
        self.frames = {r: torch.empty(E, frame_bytes, dtype=torch.uint8, device=dev) for r in self.sources}
        self.meta = {r: torch.empty(E, META_COLS, dtype=torch.int32, device=dev) for r in self.sources}

    def post(self) -> None:
        for r in self.sources:
            self.works.append(dist.irecv(self.frames[r], r, group=self.group))
            self.works.append(dist.irecv(self.meta[r], r, group=self.group))

    def take(self, device):
        """Wait for the posted packets; returns {rank: (frames, meta)} on ``device``."""
        self.wait()
        return {r: (self.frames[r].to(device, non_blocking=True), self.meta[r].to(device, non_blocking=True))
                for r in self.sources}
