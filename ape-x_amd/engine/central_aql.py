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

Transports: ``ipc`` (above; the default on GPUs) or ``p2p`` -- the torch.distributed packet
links of parallel/experience.py (RCCL send/recv, or host-staged gloo), which the bench's
preflight selects when peer access or the IPC round trip fails.  A p2p packet is the same
structure-of-arrays float block, carried as the link's byte payload; rank 0 applies the
landed packets between iterations (ring append + max-priority leaves + the step gate, the
IPC ingest's semantics) before replaying the SGD graph.

Cadence: an *iteration* of the reference is one recorded batch -- ``record_batch`` over all
workers, then ``total_ep // batch`` SGD steps (AQL_dis.py:112-129).  The learner here spins
faster than the actors deliver (a spin with nothing ingested runs no SGD step), so the
reference cadences -- target sync every ``target_update_interval`` iterations, beta
annealing, ``max_step`` -- count *recorded batches*: R packets that reached the replay
(one per actor link), read from the host-visible consumed counters the ingest publishes
(ipc) or the host's applied counts (p2p), never from learner spins.
"""
from __future__ import annotations

import copy
import time

import torch
import torch.distributed as dist

from ..parallel.experience import META_COLS, STOP, ActorLink, Dropped, LearnerLinks, engine_nonce, link_groups
from ..parallel.ipc import IpcActorLink, IpcLearnerLinks, aql_packet_floats, aql_packet_views
from .aql import AQLEngine, AQLEngineConfig, target_sync_due


class CentralAQLEngine:
    def __init__(self, cfg: AQLEngineConfig, device, rank: int | None = None, world: int | None = None,
                 depth: int = 3, dead_after: float = 30.0, heartbeat_every: float = 0.5, paced: bool = True,
                 transport: str = "auto"):
        self.device = torch.device(device)
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        if self.world < 2:
            raise ValueError("the central AQL topology needs >= 2 ranks (rank 0 learner, ranks 1.. actors)")
        self.R, self.E = self.world - 1, int(cfg.n_envs)
        self.is_learner = self.rank == 0
        if transport == "auto":
            transport = "ipc" if self.device.type == "cuda" else "p2p"
        if transport not in ("ipc", "p2p"):
            raise ValueError("transport must be ipc | p2p | auto")
        self.transport = transport
        self.depth = int(depth)
        # p2p: collective, every rank creates every link's two groups (ipc needs none)
        self.groups = link_groups(self.world) if transport == "p2p" else None
        self.store = dist.distributed_c10d._get_default_store()
        self.prefix = engine_nonce(self.store)  # collective
        self.iterations = self.learner_steps = self.actor_steps = 0
        self.spins = 0          # learner spins (ingest + gated SGD graph), >= iterations
        self._iter_base = 0     # iterations restored from a checkpoint
        self._pk0 = 0           # packets consumed before learning started (the fill)
        self._paced = bool(paced)
        self._step_base = 0
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
            if transport == "ipc":
                self.links = IpcLearnerLinks.for_aql(self.R, depth, self.E, self.pub.numel(), self.eng.replay,
                                                     self.store, self.prefix, self.device, cap=1 if paced else None,
                                                     dead_after=dead_after,
                                                     gate=(self.budget, self.gate, cfg.batch_size, self.K))
            else:
                rp = self.eng.replay
                self.row_floats = 2 * rp.obs + rp.T * rp.adim + 3
                fb = 4 * self.row_floats
                self.rx_frames = torch.empty(self.R, depth, self.E, fb, dtype=torch.uint8, device=self.device)
                self.rx_meta = torch.empty(self.R, depth, self.E, META_COLS, dtype=torch.int32, device=self.device)
                self.links = LearnerLinks(self.world, self.groups, self.store, self.pub, self.rx_frames, self.rx_meta,
                                          self._apply_p2p, dead_after, prefix=self.prefix)
                self._rows_new = 0  # rows applied since the last gate update (host count)
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
            if transport == "ipc":
                self.link = IpcActorLink(self.rank, self.store, self.prefix, self.pub, self.pkt, self.device,
                                         heartbeat_every)
            else:  # the packet's bytes are the link payload; meta column 13 >= 0 marks a real packet
                self.pkt_bytes = self.pkt.view(torch.uint8).view(self.E, -1)
                self.pkt_meta = torch.zeros(self.E, META_COLS, dtype=torch.int32, device=self.device)
                self.link = ActorLink(self.rank, self.groups[self.rank], self.store, self.pub, self.E,
                                      self.pkt_bytes.shape[1], depth, heartbeat_every, prefix=self.prefix)
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
        if self.transport == "p2p" and (self.link.stopped or self.link.check_dropped()):
            return False
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
        if self.transport == "p2p":
            try:
                self.link.push(self.pkt_bytes, self.pkt_meta)  # credit window: blocks with `depth` unconsumed
            except Dropped:
                return False
        elif not self.link.push():
            return False
        self.actor_steps += 1
        return True

    # ------------------------------------------------------------------ learner rank
    def _apply_p2p(self, ready: list[tuple[int, int]]) -> None:
        """p2p: the landed packets, in (link, packet) order, appended to the replay ring at its
        cursor + their leaves at the running max priority (the IPC ingest's ipc_apply_aql_k /
        tree write, as stream-ordered torch ops on the learner stream)."""
        e, rp, E = self.eng, self.eng.replay, self.E
        n = len(ready)
        idx = torch.tensor([(r - 1) * self.depth + k for r, k in ready], dtype=torch.int64, device=self.device)
        pk = self.rx_frames.view(self.R * self.depth, -1).index_select(0, idx).view(torch.float32).view(n, -1)
        obs, TA = rp.obs, rp.T * rp.adim
        o = [0, E * obs, 2 * E * obs, 2 * E * obs + E * TA, 2 * E * obs + E * TA + E, 2 * E * obs + E * TA + 2 * E]
        st = pk[:, o[0]:o[1]].reshape(n * E, obs)
        st2 = pk[:, o[1]:o[2]].reshape(n * E, obs)
        amu = pk[:, o[2]:o[3]].reshape(n * E, rp.T, rp.adim)
        act = pk[:, o[3]:o[4]].contiguous().view(torch.int32).reshape(n * E)
        rew = pk[:, o[4]:o[5]].reshape(n * E)
        done = pk[:, o[5]:o[5] + E].reshape(n * E)
        slots = (rp.filled + torch.arange(n * E, dtype=torch.int64, device=self.device)) % rp.capacity
        rp.st.index_copy_(0, slots, st)
        rp.st2.index_copy_(0, slots, st2)
        rp.a_mu.index_copy_(0, slots, amu)
        rp.action.index_copy_(0, slots, act)
        rp.reward.index_copy_(0, slots, rew)
        rp.done.index_copy_(0, slots, done)
        rp.filled.add_(n * E)
        s32 = slots.to(torch.int32)
        for k in range(0, s32.numel(), 1024):  # unique ring-ordered slots, <= 1024 per write
            part = s32[k:k + 1024]
            e.hip.per_write_leaves(rp.tree, part.data_ptr(), 0, part.numel(), rp.alpha, rp.max_prio.data_ptr(), 0, 0,
                                   0, 0, 0, 0, torch.cuda.current_stream(self.device).cuda_stream)
        self._rows_new += n * E

    def _p2p_gate(self) -> None:
        """p2p: the SGD steps this iteration's applied rows pay for (ipc_release_k's gate,
        carry kept in ``budget``), set before the gated SGD graph replays."""
        b = self.budget + self._rows_new
        g = torch.clamp(b // self.cfg.batch_size, max=self.K)
        self.budget.copy_(b - g * self.cfg.batch_size)
        self.gate.copy_(g.to(torch.int32))
        self._rows_new = 0

    def _ingest(self, drain: bool = False) -> None:
        if self.transport == "ipc":
            self.links.ingest(drain=drain)
        else:
            self.links.ingest(None if drain or not self._paced else 1)

    def _packets_consumed(self) -> int:
        """Packets that reached the replay so far, without a device sync: the host-visible
        per-link consumed words the IPC ingest publishes (a lower bound while the GPU runs
        behind the host), or the host's own applied counts (p2p)."""
        if self.transport == "ipc":
            return int(sum(int(c) for c in self.links.ctrl.view("consumed")))
        return int(sum(self.links.applied.values()))

    def _learner_body(self) -> None:
        if self.transport == "ipc":
            self.links.ingest()               # <= 1 packet per live link (paced) -> ring + leaves + gate
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
            self._ingest(drain=True)
            torch.cuda.synchronize(self.device)
            self.links.check_heartbeats()
            time.sleep(0.0005)
        self.budget.zero_()  # the warm-up rows pay for no SGD step (learning starts now)
        if self.transport == "p2p":
            self._rows_new = 0
        self._pk0 = self._packets_consumed()

    def capture(self) -> None:
        """hipGraph of the compute body (actor: one acting step into the packet; rank 0:
        ingest + K learner steps).  The links stay eager around it."""
        if self.is_learner:
            if self.transport == "p2p":
                self._ingest()
                self._p2p_gate()
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

    def data_iterations(self) -> int:
        """Reference iterations completed: recorded batches of R packets that reached the
        replay since learning started (+ those restored from a checkpoint)."""
        return self._iter_base + max(0, self._packets_consumed() - self._pk0) // self.R

    def _after_iteration(self) -> None:
        e = self.eng
        done = max(self.iterations, self.data_iterations())
        # the reference syncs after the SGD loop of every iteration i with i % ti == 0
        # (iteration 0 included): once per spin that completed such an iteration
        due = [i for i in range(self.iterations, done) if target_sync_due(self.cfg, i, 0, 0)]
        if due:  # (two due iterations completed in one spin: one copy serves both)
            e.learner.sync_target()
            e.target_syncs.extend(due)
        self._pack_params()  # set_worker_weights every iteration (AQL_dis.py:115), conflated
        self.links.publish(self.pub)
        self.links.check_heartbeats()
        self.spins += 1
        self.iterations = done
        # beta anneals over recorded batches (host beta, set before each spin); rank 0 never
        # acts, so its engine's fused-tail device counter is unused and needs no resync
        e._iterations = done

    def refresh_steps(self) -> int:
        """SGD steps actually taken (the device counter behind the gate: one sync) ->
        ``learner_steps``; call at log / checkpoint time."""
        self.learner_steps = self._step_base + self.sgd_steps()
        self.eng.learner_steps = self.learner_steps
        return self.learner_steps

    def restore(self, iterations: int, learner_steps: int) -> None:
        """Counters of a checkpoint (rank 0, before fill)."""
        self._iter_base = self.iterations = int(iterations)
        self._step_base = int(learner_steps) - self.sgd_steps()
        self.learner_steps = int(learner_steps)

    def iteration(self) -> bool:
        """rank 0: ingest + the gated SGD steps + publish (+ target sync); actor ranks: one
        acting step + push.  False once this rank is done."""
        if not self.is_learner:
            return self.actor_step()
        e = self.eng
        e.learner.beta.fill_(e._beta())
        if self.transport == "p2p":  # host-driven links: apply what landed, then the gate
            self._ingest()
            self._p2p_gate()
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
        return self.links.applied() if self.transport == "ipc" else dict(self.links.applied)
