"""Distributed AQL_dis across GPUs: one AQL learner fed by actor GPUs over HIP IPC
(BASELINE config 4; reference AQL_dis.py:50-53,109-126, batchrecoder_AQL.py:82-138).

The reference runs ``n_workers`` actor processes that each play episodes with a CPU copy of
the online network and hand raw ``(s, a, r, s', done, a_mu)`` transitions to the one
learner process, which inserts them at max priority, trains ``total_ep_len // batch``
SGD steps and broadcasts its weights every iteration.  Here:

* **rank 0** = the AQL learner and the one HBM replay (:class:`AQLEngine` with no acting).
  Its captured iteration graph = IPC ingest (every ready packet of every live link, paced
  at one per link: rows appended to the replay ring in (link, packet) order at its cursor,
  then one max-priority leaf write; ipc_kernels.hip ``ipc_apply_aql_k``) + up to ``K = R * E
  // batch`` fused learner steps.  The ingest turns the rows it ACTUALLY applied into a
  device step gate (carry kept): only ``(carry + rows) // batch`` of the K captured steps
  run, the others return at once -- the reference replay ratio, ``total_ep_len // batch``
  SGD steps per recorded batch (AQL_dis.py:117-118), however fast or slow the actors are.
  After each iteration it publishes ``[weights | NoisyNet eps]`` conflated over the IPC
  parameter block and syncs the target on the reference cadence.
* **ranks 1..R** = AQL actor GPUs: E vectorised envs, on-device proposal + candidate
  critic + epsilon-greedy on the global worker ladder (actor ids ``(r-1) E ..``).  One
  actor step writes its E rows straight into the packet buffer (structure of arrays, see
  ``parallel.ipc.aql_packet_views``), which one peer copy pushes into rank 0's ring under
  the credit window; new weights are pulled between steps.

Liveness, stop/drain and drop handling are the transport's (parallel/ipc.py): a dead
actor is dropped and the learner keeps training on the rest.
"""
from __future__ import annotations

import copy
import time

import torch
import torch.distributed as dist

from ..parallel.experience import STOP, engine_nonce
from ..parallel.ipc import IpcActorLink, IpcLearnerLinks, aql_packet_floats, aql_packet_views
from .aql import AQLEngine, AQLEngineConfig, target_sync_due


class CentralAQLEngine:
    def __init__(self, cfg: AQLEngineConfig, device, rank: int | None = None, world: int | None = None,
                 depth: int = 3, dead_after: float = 30.0, heartbeat_every: float = 0.5, paced: bool = True):
        self.device = torch.device(device)
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        if self.world < 2:
            raise ValueError("the central AQL topology needs >= 2 ranks (rank 0 learner, ranks 1.. actors)")
        self.R, self.E = self.world - 1, int(cfg.n_envs)
        self.is_learner = self.rank == 0
        self.store = dist.distributed_c10d._get_default_store()
        self.prefix = engine_nonce(self.store)  # collective
        self.iterations = self.learner_steps = self.actor_steps = 0
        self._g = None
        if self.is_learner:
            lc = copy.copy(cfg)
            # the reference replay ratio over everything the links can deliver per iteration
            lc.learner_steps = cfg.learner_steps or max(1, self.R * self.E // cfg.batch_size)
            if cfg.target_update_steps:
                raise ValueError("central AQL: the step gate decides the step count on the device; "
                                 "use the iteration cadence (target_update_interval)")
            depth_rows = self.R * depth * self.E
            if cfg.capacity < depth_rows:
                raise ValueError(f"central AQL: replay capacity {cfg.capacity} < links x ring depth x envs = "
                                 f"{self.R} x {depth} x {self.E} = {depth_rows} (raise --capacity or lower --n-envs)")
            self.eng = AQLEngine(lc, self.device)
            self.cfg = lc
            self.K = self.eng.K
            L = self.eng.learner
            self.pub = torch.zeros(L.P + L.eps.numel(), dtype=torch.float32, device=self.device)
            self._pack_params()
            self._broadcast_initial()
            # the step gate: rows applied -> SGD steps this iteration (carry in budget)
            self.budget = torch.zeros(1, dtype=torch.int64, device=self.device)
            self.gate = torch.zeros(1, dtype=torch.int32, device=self.device)
            self.links = IpcLearnerLinks.for_aql(self.R, depth, self.E, self.pub.numel(), self.eng.replay, self.store,
                                                 self.prefix, self.device, cap=1 if paced else None,
                                                 dead_after=dead_after,
                                                 gate=(self.budget, self.gate, cfg.batch_size, self.K))
        else:
            ac = copy.copy(cfg)
            # an actor rank keeps no replay of its own: a minimal ring, never sampled
            ac.capacity = max(2 * self.E, 64)
            ac.actor_offset, ac.total_actors = (self.rank - 1) * self.E, self.R * self.E
            ac.seed = cfg.seed + 7919 * self.rank
            self.cfg = ac
            self.eng = AQLEngine(ac, self.device)
            self.K = 0
            L = self.eng.learner
            self.pub = torch.zeros(L.P + L.eps.numel(), dtype=torch.float32, device=self.device)
            self._broadcast_initial()
            self._install_params()
            e = self.eng
            TA = e.T * e.adim
            self.pkt = torch.zeros(aql_packet_floats(self.E, e.obs, TA), dtype=torch.float32, device=self.device)
            v = aql_packet_views(self.pkt, self.E, e.obs, TA)
            self._cursor = torch.zeros(1, dtype=torch.int64, device=self.device)  # rows at 0..E-1
            self._slots = torch.zeros(self.E, dtype=torch.int32, device=self.device)
            self.into = e.hip.make_aql_insert(dict(
                st=v["st"].data_ptr(), st2=v["st2"].data_ptr(), rew=v["rew"].data_ptr(), done=v["done"].data_ptr(),
                amu=v["amu"].data_ptr(), act=v["act"].data_ptr(), C=self.E, filled=self._cursor.data_ptr(),
                slots=self._slots.data_ptr()))
            self.link = IpcActorLink(self.rank, self.store, self.prefix, self.pub, self.pkt, self.device,
                                     heartbeat_every)
            self.param_version = 0

    # ------------------------------------------------------------------ parameters
    def _pack_params(self) -> None:
        """rank 0: [online weights | NoisyNet eps] into the publish buffer (stream-ordered)."""
        L = self.eng.learner
        self.pub[:L.P].copy_(L.flat)
        self.pub[L.P:].copy_(L.eps)

    def _install_params(self) -> None:
        """actor rank: the pulled buffer -> the acting network (weights + noise)."""
        e = self.eng
        P = e.learner.P
        e.actor_flat.copy_(self.pub[:P])
        e.actor_eps.copy_(self.pub[P:])

    def _broadcast_initial(self) -> None:
        """Identical acting weights everywhere before the links start (one collective)."""
        if dist.get_backend() != "nccl":
            h = self.pub.cpu()
            dist.broadcast(h, src=0)
            if not self.is_learner:
                self.pub.copy_(h)
        else:
            dist.broadcast(self.pub, src=0)

    # ------------------------------------------------------------------ actor ranks
    def _actor_body(self) -> None:
        self.eng.actor_step(into=self.into)

    def actor_step(self) -> bool:
        """One acting step of this rank's E envs + push; False once rank 0 stopped / dropped it."""
        v = self.link.poll_params()
        if v == STOP:
            return False
        if v is not None:
            self._install_params()
            self.param_version = v
        if self._g is not None:
            self._g.replay()
        else:
            self._actor_body()
        if not self.link.push():
            return False
        self.actor_steps += 1
        return True

    # ------------------------------------------------------------------ learner rank
    def _learner_body(self) -> None:
        self.links.ingest()                   # <= 1 packet per live link (paced) -> ring + leaves + gate
        self.eng.learn_steps(gate=self.gate)  # the first gate[0] of K fused SGD steps

    def fill(self, timeout: float = 300.0) -> None:
        """rank 0: ingest until the replay holds more than ``threshold`` transitions
        (AQL_dis.py:120: learning starts once len(buffer) > batch_size)."""
        if not self.is_learner:
            return
        thr = self.cfg.threshold or self.cfg.batch_size + 1
        deadline = time.monotonic() + timeout
        while len(self.eng.replay) <= thr:
            if not self.links.live or time.monotonic() > deadline:
                raise RuntimeError(f"central AQL fill: {len(self.eng.replay)} transitions after {timeout:.0f}s, "
                                   f"live actors {sorted(self.links.live)}")
            self.links.ingest(drain=True)
            torch.cuda.synchronize(self.device)
            self.links.check_heartbeats()
            time.sleep(0.0005)
        self.budget.zero_()  # the warm-up rows pay for no SGD step (learning starts now)

    def capture(self) -> None:
        """hipGraph of the compute body (actor: one acting step into the packet; rank 0:
        ingest + K learner steps).  The links stay eager around it."""
        if self.is_learner:
            self._learner_body()  # eager warm-up: a real iteration's work
            self._after_iteration()
            torch.cuda.synchronize(self.device)
            self._g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g, capture_error_mode="thread_local"):
                self._learner_body()
        else:
            if not self.actor_step():  # eager warm-up (a real, pushed step)
                return
            torch.cuda.synchronize(self.device)
            self._g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g, capture_error_mode="thread_local"):
                self._actor_body()
        torch.cuda.synchronize(self.device)

    def sgd_steps(self) -> int:
        """SGD steps taken so far (the device step counter; one host sync)."""
        return int(self.eng.learner.step_ctr.item()) if self.is_learner else 0

    def _after_iteration(self) -> None:
        e = self.eng
        before = self.learner_steps
        self.learner_steps += self.K  # (an upper bound: the gate decides on the device, see sgd_steps)
        e.learner_steps = self.learner_steps
        if target_sync_due(self.cfg, self.iterations, before, self.learner_steps):
            e.learner.sync_target()
            e.target_syncs.append(self.iterations)
        self._pack_params()  # set_worker_weights every iteration (AQL_dis.py:115), conflated
        self.links.publish(self.pub)
        self.links.check_heartbeats()
        self.iterations += 1
        e.iterations = self.iterations

    def iteration(self) -> bool:
        """rank 0: ingest + K SGD steps + publish (+ target sync); actor ranks: one acting
        step + push.  False once this rank is done."""
        if not self.is_learner:
            return self.actor_step()
        e = self.eng
        e.learner.beta.fill_(e._beta())
        if self._g is not None:
            self._g.replay()
        else:
            self._learner_body()
        self._after_iteration()
        return True

    def close(self, timeout: float = 60.0) -> dict:
        """rank 0: stop every actor and drain its link (bounded); link stats."""
        if not self.is_learner:
            return {}
        st = self.links.close(timeout)
        torch.cuda.synchronize(self.device)
        return st

    @property
    def applied(self) -> dict:
        return self.links.applied()
