"""Global prioritized sampling over per-GPU replay shards (SURVEY §2.5, §7.4 hard part 2).

Sharded topology: every rank owns an HBM replay shard (its actor shard's experience)
and a data-parallel learner replica that samples ``B`` transitions from its own
shard -- experience never crosses xGMI.  To make the *global* update match one
prioritized buffer holding all shards, each step exchanges two numbers per shard
(total mass ``M_r`` and min priority ``pmin_r``; one 16-byte-per-rank all-gather):

* IS weights use the **global** ``pmin = min_r pmin_r``:
  ``w_i = (p_i / pmin)^-beta`` -- identical to the single-buffer weight
  ``(N P(i))^-beta / max_j (N P(j))^-beta`` because N and the total mass cancel;
* each shard's loss is scaled by ``k M_r / sum_r M_r``.  Sampling i within shard r has
  probability ``p_i / M_r``; after the DP gradient average (1/k) the expected
  gradient is ``sum_r (M_r / M) sum_{i in r} (p_i / M_r) w_i grad_i
  = sum_i (p_i / M) w_i grad_i`` -- exactly the expectation of global proportional
  sampling over the union, with fixed per-rank batch shapes (graph-capturable).

Priorities stay local (each shard updates the leaves it sampled), so no priority
routing is needed.  The exchange is a SUM all-reduce of fp32 slots [world][2] in which
each rank fills only its own slot (an all-gather in all-reduce form): the data-parallel
learner places the slots right before the conv gradients in one buffer, so the NEXT
step's exchange rides the conv-gradient all-reduce of this step (no extra collective).
The HBM replay packs its slot with one kernel from the tree root and the sampling
kernel reads the slots directly (global pmin + shard weight scale in-kernel);
``finalize()`` / ``glob`` is the generic (torch-op) form used by host replays.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class ShardedSampling:
    def __init__(self, replay, group=None, force: bool = False, slots: torch.Tensor | None = None, comm=None):
        """``slots``: fp32 [2*world] buffer to use (e.g. the learner's gradient-buffer
        prefix); ``comm``: an all-reduce with ``start(t)``/``wait(w)`` (RCCL or torch);
        default torch.distributed.  ``force``: collective even in a 1-rank group."""
        self.replay = replay
        self.group = group
        self.force = force
        self.comm = comm
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        dev = replay.device if hasattr(replay, "device") else torch.device("cpu")
        self.slots = slots if slots is not None else torch.zeros(2 * self.world, dtype=torch.float32, device=dev)
        assert self.slots.dtype == torch.float32 and self.slots.numel() == 2 * self.world
        self.glob = torch.tensor([0.0, 1.0], dtype=torch.float32, device=dev)

    def _root(self):
        return self.replay.node_sum[-1][:1], self.replay.node_min[-1][:1]

    @property
    def in_kernel(self) -> bool:
        """HBM replay: one pack kernel, and the sampler reads the slots itself."""
        return hasattr(self.replay, "pack_shard_slots")

    def sample_args(self) -> tuple:
        return self.slots, self.world, self.rank

    def pack(self) -> None:
        """slots = 0 except this rank's (mass, min priority) -- on the current stream."""
        if self.in_kernel:
            self.replay.pack_shard_slots(self.slots, self.world, self.rank)
            return
        mass, pmin = self._root()
        self.slots.zero_()
        self.slots[2 * self.rank:2 * self.rank + 1].copy_(mass)
        self.slots[2 * self.rank + 1:2 * self.rank + 2].copy_(pmin)

    def start_exchange(self):
        """Pack, then start the SUM all-reduce of the slots (the current stream does not
        wait; ``wait(work)`` joins).  Returns the work handle (None: nothing to wait)."""
        self.pack()
        if self.world == 1 and not self.force:
            return None
        if self.comm is not None:
            return self.comm.start(self.slots)
        return dist.all_reduce(self.slots, group=self.group, async_op=True)

    def wait(self, work) -> None:
        if work is None:
            return
        if self.comm is not None:
            self.comm.wait(work)
        else:
            work.wait()

    def exchange(self) -> None:
        self.wait(self.start_exchange())

    def finalize(self) -> None:
        """Device-side torch ops: glob = (global pmin, k * M_r / sum M).  Graph-capturable."""
        g = self.slots.view(self.world, 2).double()
        masses = g[:, 0]
        total = masses.sum().clamp_min(1e-300)
        self.glob[0:1].copy_(g[:, 1].min().reshape(1))
        self.glob[1:2].copy_((self.world * masses[self.rank] / total).reshape(1))

    def __call__(self) -> torch.Tensor:
        self.exchange()
        self.finalize()
        return self.glob


def global_weights_reference(shard_prios, shard_samples, beta: float):
    """Host reference of the scheme (tests): per-shard sampled priorities -> weights
    incl. the shard scale.  ``shard_prios[r]`` are all leaf priorities (p^alpha) of
    shard r, ``shard_samples[r]`` the sampled ones."""
    import numpy as np

    masses = np.array([np.sum(p) for p in shard_prios], dtype=np.float64)
    pmin = min(float(np.min(p)) for p in shard_prios)
    k = len(shard_prios)
    return [k * masses[r] / masses.sum() * (np.asarray(s, dtype=np.float64) / pmin) ** (-beta)
            for r, s in enumerate(shard_samples)]
