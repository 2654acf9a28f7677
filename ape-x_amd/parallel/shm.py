"""Versioned shared-memory parameter buffer for same-host CPU worker processes.

Replaces the reference's per-worker pickled ``state_dict`` tasks
(batchrecorder.py:140-146, batchrecoder_AQL.py:125-132: n pickles of the full model
per publish, unaddressed so a worker can miss an update) with one flat
fp32 buffer in shared memory plus a seqlock version counter:

* the publisher bumps the version to odd, copies the flat parameters, bumps to even;
* a subscriber copies only when the version is even and newer than what it holds,
  and re-checks the version after the copy (retry on a torn read).

Every worker therefore sees the newest weights ("conflate" semantics of the origin
PUB/SUB socket, origin_repo/actor.py:44) with zero pickling.
"""
from __future__ import annotations

import multiprocessing as mp

import torch


def flat_params(module: torch.nn.Module) -> torch.Tensor:
    """All parameters *and* buffers (NoisyLinear epsilons live in buffers) flattened."""
    ts = [t.detach().reshape(-1).float().cpu() for t in module.state_dict().values()]
    return torch.cat(ts) if ts else torch.zeros(0)


def load_flat_(module: torch.nn.Module, flat: torch.Tensor) -> None:
    off = 0
    with torch.no_grad():
        for t in module.state_dict().values():
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t).to(t.dtype))
            off += n
    if off != flat.numel():
        raise ValueError(f"flat buffer has {flat.numel()} values, module needs {off}")


class SharedParams:
    """Picklable handle (works with both fork and spawn start methods)."""

    def __init__(self, numel: int, ctx=None):
        ctx = ctx or mp.get_context()
        self.buf = torch.zeros(int(numel), dtype=torch.float32).share_memory_()
        self.version = ctx.Value("q", 0, lock=False)

    @classmethod
    def for_module(cls, module: torch.nn.Module, ctx=None) -> "SharedParams":
        sp = cls(flat_params(module).numel(), ctx)
        return sp

    # -- publisher -------------------------------------------------------------
    def publish(self, module_or_flat) -> int:
        flat = module_or_flat if isinstance(module_or_flat, torch.Tensor) else flat_params(module_or_flat)
        v = self.version.value
        self.version.value = v + 1          # odd: write in progress
        self.buf.copy_(flat.reshape(-1).cpu())
        self.version.value = v + 2          # even: consistent
        return (v + 2) // 2

    # -- subscriber ------------------------------------------------------------
    def published(self) -> int:
        return self.version.value // 2

    def pull(self, module: torch.nn.Module, have: int) -> int:
        """Load the newest weights into ``module`` if newer than ``have``; returns the
        version now held."""
        for _ in range(100):
            v0 = self.version.value
            if v0 % 2 or v0 // 2 <= have:
                if v0 % 2 == 0:
                    return have
                continue
            snap = self.buf.clone()
            if self.version.value == v0:
                load_flat_(module, snap)
                return v0 // 2
        return have
