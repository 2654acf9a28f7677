"""Data-parallel learner replicas: one flat-gradient all-reduce per step.

The reference has a single learner GPU (learner.py:139) and no collectives.  For the
sharded topology (one actor shard + replay shard + learner replica per GPU) the
gradient of the whole 0.88M-parameter network lives in ONE contiguous fp32 buffer
(DuelingDQN.flatten_parameters), so a step needs exactly one 3.5 MB all-reduce --
on xGMI's point-to-point links a single large ring/tree collective beats per-tensor
buckets (each per-link bound; fewer, larger messages).  With the ``nccl`` backend
this is RCCL over xGMI; with ``gloo`` it runs on CPU for tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class FlatGradAllReduce:
    """Flat-gradient all-reduce across the process group.

    ``__call__(flat)`` averages in place (synchronous w.r.t. the current stream).  The
    learner uses the split, asynchronous form instead: ``start(t)`` enqueues an RCCL SUM
    of ``t`` on the process group's own stream and returns at once (the current stream
    does NOT wait), ``wait(*works)`` makes the current stream wait for them, and the
    optimizer applies the 1/world mean (``grad_scale``) -- so the FC1/head slice's
    all-reduce overlaps the conv backward, and no scaling kernel runs.
    """

    def __init__(self, world_size: int | None = None, group=None, bucket_bytes: int | None = None,
                 force: bool = False):
        """``force``: issue the collectives even in a 1-rank group (measures the RCCL call
        path and host cost of the data-parallel step on a single GPU)."""
        self.group = group
        self.force = force
        self.world = world_size or dist.get_world_size(group)
        self.scale = 1.0 / self.world
        self.bucket_elems = None if bucket_bytes is None else max(1, bucket_bytes // 4)

    def __call__(self, flat: torch.Tensor) -> None:
        if self.world == 1:
            return
        if self.bucket_elems is None or flat.numel() <= self.bucket_elems:
            dist.all_reduce(flat, group=self.group)
        else:  # optional bucketing (e.g. to overlap with a backward in flight)
            for off in range(0, flat.numel(), self.bucket_elems):
                dist.all_reduce(flat[off:off + self.bucket_elems], group=self.group)
        flat.mul_(self.scale)

    def start(self, t: torch.Tensor):
        """Asynchronous in-place SUM of ``t``; returns the work handle(s) (None: world 1)."""
        if self.world == 1 and not self.force:
            return None
        if self.bucket_elems is None or t.numel() <= self.bucket_elems:
            return dist.all_reduce(t, group=self.group, async_op=True)
        return [dist.all_reduce(t[off:off + self.bucket_elems], group=self.group, async_op=True)
                for off in range(0, t.numel(), self.bucket_elems)]

    @staticmethod
    def wait(*works) -> None:
        """Current stream waits for the given start() handles (no host block on RCCL)."""
        for w in works:
            if w is None:
                continue
            for x in (w if isinstance(w, list) else [w]):
                x.wait()


def allreduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
        t.div_(dist.get_world_size(group))
    return t
