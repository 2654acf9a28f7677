"""Learner -> actor parameter publication.

Reference: the learner pickles ``state_dict()`` (3.5 MB), copies it to the CPU and
sends it on a ZeroMQ PUB socket with HWM 3 every 25 steps; actors SUB with
CONFLATE=1 (only the newest version matters) and poll every 400 actor steps
(learner.py:57-68,169-170; actor.py:40-49,97-103).

Here the parameters are one flat fp32 device buffer and publication is a single
RCCL broadcast over xGMI (``torch.distributed`` ``nccl`` backend), tagged with a
version counter so subscribers can tell fresh from stale and conflate (keep only the
newest).  ``ParamPublisher``/``ParamSubscriber`` are the versioned, double-buffered
pair; ``broadcast_flat`` is the plain collective (also used to give DP replicas
identical initial weights).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def broadcast_flat(flat: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)
    return flat


class ParamPublisher:
    """Rank ``src`` publishes its flat params to every rank of ``group``.

    Collective semantics: every rank calls ``publish()`` at the same learner-step
    cadence; the payload is [version, params...] so a receiver knows which learner
    step its weights come from.  Double buffering: the broadcast lands in a staging
    buffer on the comm stream; ``ParamSubscriber.maybe_swap`` copies it into the live
    actor weights only when a newer version has arrived (CONFLATE semantics).
    """

    def __init__(self, flat: torch.Tensor, src: int = 0, group=None, stream: torch.cuda.Stream | None = None):
        self.flat = flat
        self.src = src
        self.group = group
        self.version = 0
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.staging = torch.empty(flat.numel() + 1, dtype=torch.float32, device=flat.device)
        self.stream = stream
        self.event = None

    def publish(self, version: int | None = None) -> None:
        self.version = self.version + 1 if version is None else int(version)
        if self.rank == self.src:
            self.staging[0].fill_(float(self.version))
            self.staging[1:].copy_(self.flat)
        if self.stream is not None and self.flat.is_cuda:
            self.stream.wait_stream(torch.cuda.current_stream(self.flat.device))
            with torch.cuda.stream(self.stream):
                broadcast_flat(self.staging, self.src, self.group)
                self.event = torch.cuda.Event()
                self.event.record(self.stream)
        else:
            broadcast_flat(self.staging, self.src, self.group)


class ParamSubscriber:
    def __init__(self, publisher: ParamPublisher, live_flat: torch.Tensor):
        self.pub = publisher
        self.live = live_flat
        self.version = -1

    def maybe_swap(self) -> bool:
        """Adopt the newest published params if newer than what we hold (returns True if swapped)."""
        if self.pub.event is not None:
            torch.cuda.current_stream(self.live.device).wait_event(self.pub.event)
        v = int(self.pub.staging[0].item())
        if v > self.version:
            self.live.copy_(self.pub.staging[1:])
            self.version = v
            return True
        return False
