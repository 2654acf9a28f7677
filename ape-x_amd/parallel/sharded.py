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
routing is needed.  ``exchange()`` is the eager collective (before the learner
graph); ``finalize()`` is captured inside the learner graph and writes ``glob`` =
(global pmin, weight scale) for the sampling kernel.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class ShardedSampling:
    def __init__(self, replay, group=None, force: bool = False):
        self.replay = replay
        self.group = group
        self.force = force  # collective even in a 1-rank group (single-GPU measurement of the DP path)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        dev = replay.device if hasattr(replay, "device") else torch.device("cpu")
        self.local = torch.zeros(2, dtype=torch.float64, device=dev)
        self.gathered = torch.zeros(self.world * 2, dtype=torch.float64, device=dev)
        self.glob = torch.tensor([0.0, 1.0], dtype=torch.float32, device=dev)

    def _root(self):
        return self.replay.node_sum[-1][:1], self.replay.node_min[-1][:1]

    @property
    def in_kernel(self) -> bool:
        """HBM replay: the tree kernels keep ``root_stats`` (the send buffer) current and
        the sampler reads ``gathered`` itself -- no pack copies, no finalize ops."""
        return hasattr(self.replay, "root_stats")

    def sample_args(self) -> tuple:
        return self.gathered, self.world, self.rank

    def exchange(self) -> None:
        """Pack this shard's (mass, min priority) and all-gather them (eager: collectives
        stay outside the captured graphs)."""
        self.wait(self.start_exchange())

    def start_exchange(self):
        """Asynchronous form: the pack runs on the current stream, the all-gather on the
        process group's stream without making the current stream wait -- the engine
        issues the NEXT step's exchange right after this step's backward (the tree is
        final by then) so it overlaps the optimizer.  Returns the work handle."""
        if self.in_kernel:
            local = self.replay.root_stats
        else:
            mass, pmin = self._root()
            self.local[0:1].copy_(mass)
            self.local[1:2].copy_(pmin)
            local = self.local
        if self.world > 1 or self.force:
            return dist.all_gather_into_tensor(self.gathered, local, group=self.group, async_op=True)
        self.gathered.copy_(local)
        return None

    @staticmethod
    def wait(work) -> None:
        if work is not None:
            work.wait()

    def finalize(self) -> None:
        """Device-side: glob = (global pmin, k * M_r / sum M).  Graph-capturable."""
        g = self.gathered.view(self.world, 2)
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
