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
    """Callable: average a flat gradient buffer across the process group in place."""

    def __init__(self, world_size: int | None = None, group=None, bucket_bytes: int | None = None):
        self.group = group
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


def allreduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
        t.div_(dist.get_world_size(group))
    return t
