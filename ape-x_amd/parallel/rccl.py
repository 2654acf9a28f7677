"""Direct RCCL communicator for the data-parallel learner.

``torch.distributed`` (backend "nccl" = RCCL on ROCm) remains the control plane:
rendezvous, the one-off weight broadcast and the ncclUniqueId hand-off.  The per-step
gradient traffic goes through a communicator of our own (``_apex_hip.rccl_*``, a thin
C++ wrapper over ncclCommInitRank / ncclAllReduce), enqueued on a comm stream this
module owns with plain HIP events for ordering.  Measured on MI355X with roctx ranges,
a torch async collective costs ~30 us of host time (work objects, watchdog, stream
hops); the learner step is ~0.3 ms, so that overhead made the data-parallel step
host-bound.  The direct call costs a few microseconds.

The interface matches ``parallel.dp.FlatGradAllReduce`` (``start`` / ``wait``; SUM, the
optimizer applies 1/world), so the engine and the shard-mass exchange use either.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops

_DT = {torch.float32: "f32", torch.float64: "f64", torch.bfloat16: "bf16", torch.int64: "i64", torch.uint8: "u8"}


class RcclComm:
    """One RCCL communicator over the ranks of ``group`` (default: the world)."""

    def __init__(self, device, group=None):
        self.hip = ops.hip()
        self.device = torch.device(device)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        root = dist.get_global_rank(group, 0) if group is not None else 0
        box = [self.hip.rccl_unique_id() if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=root, group=group, device=self.device)
        self.handle = self.hip.rccl_comm_init(box[0], self.world, self.rank, self.device.index or 0)

    def count(self) -> int:
        """Ranks RCCL itself reports for this communicator (ncclCommCount)."""
        return int(self.hip.rccl_comm_count(self.handle))

    def all_reduce_sum(self, t: torch.Tensor, stream) -> None:
        assert t.is_contiguous() and t.device == self.device
        self.hip.rccl_all_reduce_sum(t.data_ptr(), t.numel(), _DT[t.dtype], self.handle, stream.cuda_stream)

    def broadcast(self, t: torch.Tensor, root: int, stream) -> None:
        assert t.is_contiguous() and t.device == self.device
        self.hip.rccl_broadcast(t.data_ptr(), t.numel(), _DT[t.dtype], root, self.handle, stream.cuda_stream)

    def close(self) -> None:
        if self.handle:
            self.hip.rccl_comm_destroy(self.handle)
            self.handle = 0


class RcclGradAllReduce:
    """Asynchronous in-place SUM all-reduces on a dedicated comm stream.

    ``start(t)`` -> the comm stream waits for the caller's stream, the all-reduce is
    enqueued there, an event marks its end (returned); ``wait(*events)`` makes the
    caller's stream wait.  Events come from a small ring (re-recording an event after
    the waits on it were enqueued is safe)."""

    def __init__(self, device, group=None, force: bool = False, comm: RcclComm | None = None):
        self.device = torch.device(device)
        self.comm = comm or RcclComm(self.device, group)
        self.world = self.comm.world
        self.force = force
        self.scale = 1.0 / self.world
        self.stream = torch.cuda.Stream(device=self.device)
        self._ring = [torch.cuda.Event() for _ in range(16)]
        self._k = 0

    def _event(self):
        e = self._ring[self._k]
        self._k = (self._k + 1) % len(self._ring)
        return e

    def mark(self):
        """Record the point the next :meth:`start` depends on (``start(t, ready=...)`` may then
        be issued later: in a captured graph the chain launched in between stays the fork's
        first child and keeps the graph's queue; the collective branch takes the hand-off)."""
        if self.world == 1 and not self.force:
            return None
        ready = self._event()
        ready.record(torch.cuda.current_stream(self.device))
        return ready

    def start(self, t: torch.Tensor, ready=None):
        if self.world == 1 and not self.force:
            return None
        if ready is None:
            ready = self.mark()
        self.stream.wait_event(ready)
        self.comm.all_reduce_sum(t, self.stream)
        done = self._event()
        done.record(self.stream)
        return done

    def wait(self, *events) -> None:
        cur = torch.cuda.current_stream(self.device)
        for e in events:
            if e is not None:
                cur.wait_event(e)

    def __call__(self, flat: torch.Tensor) -> None:
        """Synchronous mean (the FlatGradAllReduce call form)."""
        self.wait(self.start(flat))
        if self.world > 1 or self.force:
            flat.mul_(self.scale)
