"""Central-replay Ape-X topology across GPUs, asynchronous and fault tolerant
(BASELINE config 3).

Rank 0 is the learner and holds the one HBM replay (frame ring + transition table +
priority tree), split into one region per actor rank.  Ranks 1..W-1 are actor GPUs:
each runs an :class:`ActorShard` (E GPU envs, batched inference with the global Ape-X
epsilon ladder, on-device n-step) writing into a *local mirror* of its region, and pushes
every actor step (E new frames + E transition rows) to rank 0 over its own link
(``parallel.experience``; RCCL over xGMI with ``nccl``, host-staged with ``gloo``).

Nothing is lock-step (the reference decouples its roles the same way: actor.py pushes with
3 outstanding, replay.py ingests with 16 workers, learner.py prefetches):

* actor rank: act (hipGraph) -> copy the packet into a free slot of its send ring (credit
  window of ``depth`` = 3 packets in flight, actor.py:105-115) -> isend; between steps it
  polls its parameter subscription (conflated + versioned, actor.py:40-49) and posts a
  heartbeat to the TCPStore;
* rank 0: learner step (hipGraph) -> poll every live link's pre-posted receives without
  blocking -> ONE batched scatter of all landed packets into their regions + one tree
  write (``apply_packets``) on the learner stream -> re-post; every
  ``publish_param_interval`` steps a new parameter version to every link whose previous
  one was delivered.  The learner never waits for an actor: a slow actor only lowers the
  experience rate, a dead one (receive error or a heartbeat that stopped for
  ``dead_after`` s) is dropped and the learner keeps stepping on the rest
  (learner.py:57-68: PUB/SUB drops slow subscribers).
* :meth:`close` ends the run with a bounded handshake (stop on the parameter channel,
  packet counts through the store, filler packets) so no send or receive is left posted.

``APEX_FAULT=actor<r>:kill@<step>`` hard-kills actor rank r at that actor step (tests).
"""
from __future__ import annotations

import dataclasses
import time
from types import SimpleNamespace

import torch
import torch.distributed as dist

from ..models.dqn import DuelingDQN
from ..models.fused import make_hip_net, make_workspace
from .. import ops
from ..parallel.experience import (META_COLS, STOP, ActorLink, Dropped, LearnerLinks, Region, apply_packets,
                                   engine_nonce, link_groups)
from ..parallel.ipc import IpcActorLink, IpcLearnerLinks, packet_bytes
from ..roles.common import maybe_fault
from .actor_shard import ActorShard
from .apex import EngineConfig
from .hbm_replay import FRAME_BYTES, HBMReplay
from .learner import DQNLearner


def stage_packet(hip, replay: HBMReplay, actor: ActorShard, packet: torch.Tensor, E: int, initial: bool = False):
    """ipc_stage_dqn over an actor shard's local replay mirror into ``packet`` (current stream)."""
    rp, a = replay, actor
    d = dict(frames=rp.frames.data_ptr(), new_frame=a.new_frame.data_ptr(), packet=packet.data_ptr(), E=E,
             initial=int(initial))
    if initial:
        d.update(hist=a.st["hist"].data_ptr(), actions=a.actions.data_ptr())
    else:
        d.update(s_ids=rp.s_ids.data_ptr(), s2_ids=rp.s2_ids.data_ptr(), action=rp.action.data_ptr(),
                 reward=rp.reward.data_ptr(), done=rp.done.data_ptr(), slot=a.slot.data_ptr(), prio=a.prio.data_ptr())
    hip.ipc_stage_dqn(d, torch.cuda.current_stream().cuda_stream)


def build_actor_rank(cfg: EngineConfig, device, rank: int, R: int, C_r: int, F_r: int,
                     model: DuelingDQN | None = None) -> SimpleNamespace:
    """An actor GPU's state (central topology rank ``rank`` of R actor ranks): the local
    replay mirror of its region (frame ring + transition rows, no sampling), the
    :class:`ActorShard` on the global epsilon ladder, the acting network (packed HIP copy of
    ``model``) and its workspace."""
    lc, E = cfg.learner, cfg.n_envs
    replay = HBMReplay(C_r, E, lc.n_step, cfg.alpha, device, frame_capacity=F_r, exact_mass=cfg.exact_mass,
                       seed=cfg.seed + rank)
    actor = ActorShard(replay, E, cfg.n_actions, lc.n_step, lc.gamma, cfg.eps_base, cfg.eps_alpha,
                       actor_offset=(rank - 1) * E, total_actors=R * E, seed=cfg.seed + 7919 * rank,
                       mode=cfg.nstep_mode)
    model = (model if model is not None else DuelingDQN.from_shapes((4, 84, 84), cfg.n_actions)).to(device)
    flat = model.flatten_parameters()
    for p in model.parameters():
        p.requires_grad_(False)
    net = make_hip_net(model, lc.dtype)
    ws = make_workspace(E, cfg.n_actions, device, lc.dtype)
    ws.q = actor.q  # the heads kernel writes Q (and picks the actions) in place
    return SimpleNamespace(replay=replay, actor=actor, model=model, flat=flat, net=net, ws=ws, E=E)


def actor_rank_step(hip, a, packet: torch.Tensor) -> None:
    """One actor step of an actor rank's E envs into its packet (``a``: :func:`build_actor_rank`
    fields): the forward (conv1 reads the stacks from the local frame ring; the heads kernel
    writes Q and picks the eps-greedy actions), env step + n-step rows into the local mirror
    (no local tree: the priorities travel with the rows), then the one staging launch."""
    a.net(a.replay.frames, a.ws, a.actor.st["hist"], act=a.actor.act_args())
    a.actor.act_and_step(None, selected=True, tree=False)
    stage_packet(hip, a.replay, a.actor, packet, a.E)


def region_geometry(cfg: EngineConfig, n_actor_ranks: int) -> tuple[int, int]:
    """(transition slots, frame slots) per actor-rank region; multiples of the env count."""
    E, n = cfg.n_envs, cfg.learner.n_step
    c = max(E, (cfg.replay_capacity // max(1, n_actor_ranks)) // E * E)
    f = c + -(-(2 * n + 8) * E // E) * E
    return c, f


class CentralApexEngine:
    def __init__(self, cfg: EngineConfig, device, rank: int | None = None, world: int | None = None,
                 depth: int = 3, dead_after: float = 30.0, heartbeat_every: float = 0.5, paced: bool = True,
                 transport: str = "auto", emulate_links: int = 0):
        """``transport``: "ipc" (HIP IPC rings in rank 0's HBM, parallel/ipc.py; the default on
        GPUs), "p2p" (torch.distributed isend/irecv links, parallel/experience.py; CPU tests and
        the host-staged gloo rehearsal) or "auto".  ``emulate_links`` = R > 0: THIS process is
        rank 0 of a virtual world of R + 1 whose R actor links are emulated in-process
        (parallel.ipc.EmulatedActorLinks: synthetic packets written into the real IPC ring,
        ingested by the real in-graph ingest) -- the central learner's load at N = R + 1 GPUs,
        measured on one."""
        self.cfg = cfg
        self.hip = ops.hip()
        self.device = torch.device(device)
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        self.emu = None
        if emulate_links:
            if dist.get_world_size() != 1 or transport not in ("ipc", "auto"):
                raise ValueError("emulate_links: one process (a world-1 process group) over the IPC transport")
            self.rank, self.world = 0, int(emulate_links) + 1
        if self.world < 2:
            raise ValueError("the central topology needs >= 2 ranks (rank 0 learner, ranks 1.. actors)")
        self.R = self.world - 1
        self.depth = int(depth)
        lc = cfg.learner
        E = cfg.n_envs
        self.E = E
        self.C_r, self.F_r = region_geometry(cfg, self.R)
        torch.manual_seed(cfg.seed)
        model = DuelingDQN.from_shapes((4, 84, 84), cfg.n_actions)
        self.is_learner = self.rank == 0
        self.learn_steps = self.actor_steps = 0
        self._g_actor = self._g_learn = None
        if transport == "auto":
            transport = "ipc" if self.device.type == "cuda" else "p2p"
        if transport not in ("ipc", "p2p"):
            raise ValueError("transport must be ipc | p2p | auto")
        self.transport = transport
        # p2p: collective, every rank creates every link's two groups (ipc needs none)
        self.groups = link_groups(self.world) if transport == "p2p" else None
        self.store = dist.distributed_c10d._get_default_store()
        self.prefix = engine_nonce(self.store)  # collective: per-engine store-key namespace
        self.heartbeat_every = float(heartbeat_every)  # seconds between actor heartbeats
        # paced: each learner step consumes at most actor_steps_per_learner_step packets per link,
        # so the 3-packet credit window holds every actor at that rate (the single-GPU engine's
        # ratio); unpaced: actors run free and rank 0 ingests everything that landed
        self.ingest_cap = cfg.actor_steps_per_learner_step if paced else None
        if self.is_learner:
            self.replay = HBMReplay(self.C_r * self.R, E, lc.n_step, cfg.alpha, self.device,
                                    frame_capacity=self.F_r * self.R, exact_mass=cfg.exact_mass, seed=cfg.seed)
            if transport in ("ipc", "auto") and self.device.type == "cuda" and lc.forward == "hip":
                # the IPC ingest runs on the learner's tree stream beside the backward: the step
                # reads private copies of its sampled rows (the ingest may rewrite their slots)
                lc = dataclasses.replace(lc, private_rows=True)
            self.learner = DQNLearner(model, self.replay, lc)
            self.flat = self.learner.flat
            self.regions = {r: Region((r - 1) * self.C_r, self.C_r, (r - 1) * self.F_r, self.F_r)
                            for r in range(1, self.world)}
            rp = self.replay
            self.tables = {"frames": rp.frames, "s_ids": rp.s_ids, "s2_ids": rp.s2_ids, "action": rp.action,
                           "reward": rp.reward, "done": rp.done}
        else:
            a = build_actor_rank(cfg, self.device, self.rank, self.R, self.C_r, self.F_r, model)
            self.replay, self.actor, self.model, self.flat, self.net, self.ws = (a.replay, a.actor, a.model, a.flat,
                                                                                 a.net, a.ws)
        self._initial_params()
        if self.is_learner:
            self._setup_learner_links(dead_after)
            if emulate_links:
                from ..parallel.ipc import EmulatedActorLinks

                self.emu = EmulatedActorLinks(self.links, self.C_r, self.F_r, cfg.n_actions, seed=cfg.seed)
                self._estream = torch.cuda.Stream(device=self.device)
                self._ev_step = torch.cuda.Event()  # the previous learner step (its ingest freed credit)
                self._ev_step.record(torch.cuda.current_stream(self.device))
        else:
            self._setup_actor_link()

    # ------------------------------------------------------------------ setup
    def _emu_push(self) -> None:
        """Emulated links: every link's next packet, on the emulators' own stream, after the
        previous learner step (whose ingest returned the credit) -- a paced actor pushes as
        soon as its credit window opens, so each link delivers one packet per learner step."""
        if self.emu is not None:
            self._estream.wait_event(self._ev_step)
            with torch.cuda.stream(self._estream):
                self.emu.push()

    def _initial_params(self) -> None:
        """Identical weights everywhere before the links start (one collective broadcast)."""
        if dist.get_world_size() == 1:
            return
        if dist.get_backend() != "nccl":
            h = self.flat.cpu()
            dist.broadcast(h, src=0)
            if not self.is_learner:
                self.flat.copy_(h)
        else:
            dist.broadcast(self.flat, src=0)
        if not self.is_learner:
            self.net.repack()

    def _setup_learner_links(self, dead_after: float) -> None:
        R, D, E, dev = self.R, self.depth, self.E, self.device
        if self.transport == "ipc":
            self.links = IpcLearnerLinks.for_dqn(R, D, E, self.flat.numel(), self.replay, self.regions, self.store,
                                                 self.prefix, dev, cap=self.ingest_cap, dead_after=dead_after)
            return
        self.rx_frames = torch.empty(R, D, E, FRAME_BYTES, dtype=torch.uint8, device=dev)
        self.rx_meta = torch.empty(R, D, E, META_COLS, dtype=torch.int32, device=dev)
        # per receive slot (link r, ring slot k): the region's frame / transition-slot base
        fb = [self.regions[r].frame_base for r in range(1, self.world) for _ in range(D)]
        sb = [self.regions[r].slot_base for r in range(1, self.world) for _ in range(D)]
        self._fbase = torch.tensor(fb, dtype=torch.int64, device=dev)
        self._sbase = torch.tensor(sb, dtype=torch.int64, device=dev)
        self.links = LearnerLinks(self.world, self.groups, self.store, self.flat, self.rx_frames, self.rx_meta,
                                  self._apply, dead_after, prefix=self.prefix)
        # packet-selection index ring: pinned once, reused after its previous H2D copy completed
        self._sel_host = [torch.empty(R * D, dtype=torch.int64).pin_memory() for _ in range(4)]
        self._sel_ev = [None] * 4
        self._sel_k = 0

    def _setup_actor_link(self) -> None:
        # one contiguous packet (E frames | E x 14 meta) that ONE staging launch fills per actor step
        E, FB = self.E, FRAME_BYTES
        self.pkt = torch.empty(packet_bytes(E), dtype=torch.uint8, device=self.device)
        self.pkt_frames = self.pkt[:E * FB].view(E, FB)
        self.pkt_meta = self.pkt[E * FB:].view(torch.int32).view(E, META_COLS)
        self.param_version = 0
        if self.transport == "ipc":
            self.link = IpcActorLink(self.rank, self.store, self.prefix, self.flat, self.pkt, self.device,
                                     self.heartbeat_every)
            self._stage_packet(initial=True)  # the reset frames are the first packet
            self.link.push()
            return
        self.link = ActorLink(self.rank, self.groups[self.rank], self.store, self.flat, self.E, FRAME_BYTES,
                              self.depth, self.heartbeat_every, prefix=self.prefix)
        self._stage_packet(initial=True)  # the reset frames are the first packet
        self.link.push(self.pkt_frames, self.pkt_meta)

    @property
    def stopped(self) -> bool:
        return self.link.stopped

    @property
    def live(self) -> set:
        return self.links.live

    @property
    def dropped(self) -> dict:
        return self.links.dropped

    @property
    def applied(self) -> dict:
        """Packets applied per actor rank (ipc: device counters, one host sync)."""
        return self.links.applied() if self.transport == "ipc" else self.links.applied

    # ------------------------------------------------------------------ actor ranks
    def _stage_packet(self, initial: bool = False) -> None:
        """The actor step's packet in ONE launch (ipc_kernels.hip ipc_stage_dqn_k): the E new
        frames out of the local frame ring + the E rows the n-step kernel just wrote into the
        local mirror (make_batch of memory.py:466-469, actor.py:105-115).  ``initial``: the
        reset frames only, every row a filler (slot -1: no transition row is written)."""
        a, rp = self.actor, self.replay
        stage_packet(self.hip, rp, a, self.pkt, self.E, initial)

    def _actor_body(self) -> None:
        actor_rank_step(self.hip, self, self.pkt)

    def actor_step(self) -> bool:
        """One actor step + push; False once the learner has stopped or dropped this actor."""
        if self.transport == "ipc":
            return self._actor_step_ipc()
        if self.link.stopped or self.link.check_dropped():
            return False
        v = self.link.poll_params()
        if v == STOP:
            return False
        if v is not None:
            self.net.repack()
            self.param_version = v
        maybe_fault("actor", self.rank, self.actor_steps)
        if self._g_actor is not None:
            self._g_actor.replay()
        else:
            self._actor_body()
        try:
            self.link.push(self.pkt_frames, self.pkt_meta)  # credit window: blocks only with 3 unconsumed
        except Dropped:
            return False
        self.actor_steps += 1
        return True

    def _actor_step_ipc(self) -> bool:
        v = self.link.poll_params()
        if v == STOP:
            return False
        if v is not None:
            self.net.repack()
            self.param_version = v
        maybe_fault("actor", self.rank, self.actor_steps)
        if self._g_actor is not None:
            self._g_actor.replay()
        else:
            self._actor_body()
        if not self.link.push():  # credit window of ``depth`` packets; False: stopped / dropped
            return False
        self.actor_steps += 1
        return True

    # ------------------------------------------------------------------ learner rank
    def _apply(self, ready: list[tuple[int, int]]) -> None:
        """ONE batched scatter of every landed packet into its region + one tree write,
        on the learner stream (between learner steps)."""
        j = self._sel_k
        self._sel_k = (j + 1) % len(self._sel_host)
        if self._sel_ev[j] is not None:
            self._sel_ev[j].synchronize()  # (long done) this buffer's previous H2D copy
        n = len(ready)
        host = self._sel_host[j]
        for i, (r, k) in enumerate(ready):
            host[i] = (r - 1) * self.depth + k
        idx = host[:n].to(self.device, non_blocking=True)
        ev = self._sel_ev[j] = self._sel_ev[j] or torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        D, E = self.depth, self.E
        frames = self.rx_frames.view(self.R * D, E, FRAME_BYTES).index_select(0, idx)
        meta = self.rx_meta.view(self.R * D, E, META_COLS).index_select(0, idx)
        slots, prio = apply_packets(self.tables, frames, meta, self._fbase.index_select(0, idx),
                                    self._sbase.index_select(0, idx))
        # the fill counter advances by the real transition rows (filler rows, e.g. the
        # reset-frame packet's, carry frames only -- as the IPC ingest counts them)
        self.replay.filled.add_((slots >= 0).sum())
        self.replay.write_priorities(slots, prio, dedup=False)

    def ingest(self, cap: int | None = None) -> int:
        if self.transport == "ipc":  # device-side (normally captured in the learner graph)
            self.links.ingest()
            return 0
        return self.links.ingest(cap)

    def publish_params(self) -> None:
        """Conflated, versioned publish to every live actor link (rank 0)."""
        if self.is_learner:
            self.links.publish(self.flat)

    def _learner_body(self) -> None:
        if self.transport == "ipc" and self.learner.rows is not None:
            # ingest rides in the learner graph (no host poll per step), on the tree stream
            # after the step's priority write: beside the conv backward, off the critical chain
            self.learner.tree_tail.append(self.links.ingest)
            self.learner.step()
            return
        self.learner.step()
        if self.transport == "ipc":
            self.links.ingest()

    def learner_step(self) -> None:
        if self._g_learn is not None:
            self._g_learn.replay()
        else:
            self._learner_body()
        if self.emu is not None:
            self._ev_step.record(torch.cuda.current_stream(self.device))
        self.learn_steps += 1
        if self.learn_steps % self.cfg.target_update_interval == 0:
            self.learner.sync_target()

    def close(self, timeout: float = 60.0) -> dict:
        """Stop every live actor and drain its link (bounded).  Returns link stats."""
        if not self.is_learner:
            return {}
        if self.emu is not None:
            self.emu.finish()
        st = self.links.close(timeout)
        torch.cuda.synchronize(self.device)
        return st

    # ------------------------------------------------------------------ driver
    def fill(self, timeout: float = 600.0) -> None:
        """Rank 0: ingest until ``threshold_size`` transitions landed (bounded); actor
        ranks start acting in :meth:`train_step`."""
        if not self.is_learner:
            return
        need = -(-self.cfg.threshold_size // self.E)
        deadline = time.monotonic() + timeout
        if self.transport == "ipc":
            # (+ every real actor's reset-frame packet; emulated links send none)
            while sum(self.applied.values()) < need + (0 if self.emu is not None else len(self.live)):
                if not self.live or time.monotonic() > deadline:
                    raise RuntimeError(f"central fill: {sum(self.applied.values())} packets after {timeout}s, "
                                       f"live actors {sorted(self.live)}")
                self._emu_push()
                torch.cuda.synchronize(self.device)
                self.links.ingest(drain=True)
                torch.cuda.synchronize(self.device)
                self.links.check_heartbeats()
                time.sleep(0.0005)
            return
        while sum(self.applied.values()) < need + len(self.live):
            if not self.live or time.monotonic() > deadline:
                raise RuntimeError(f"central fill: {sum(self.applied.values())} packets after {timeout}s, "
                                   f"live actors {sorted(self.live)}")
            if not self.ingest():
                time.sleep(0.0005)
            self.links.check_heartbeats()

    def capture(self) -> None:
        """hipGraphs of the compute bodies (the links stay eager around them)."""
        pool = torch.cuda.graph_pool_handle()
        if self.is_learner:
            self._emu_push()
            self._learner_body()  # eager warm-up (a real step)
            self.learn_steps += 1
            torch.cuda.synchronize(self.device)
            self._g_learn = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_learn, pool=pool, capture_error_mode="thread_local"):
                self._learner_body()
        else:
            if not self.actor_step():  # eager warm-up (a real, pushed step)
                return
            torch.cuda.synchronize(self.device)
            self._g_actor = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_actor, pool=pool, capture_error_mode="thread_local"):
                self._actor_body()
        torch.cuda.synchronize(self.device)

    def train_step(self) -> bool:
        """Rank 0: one learner step + ingest (+ publish / heartbeat checks).  Actor ranks:
        ``actor_steps_per_learner_step`` actor steps.  False once this rank is done."""
        if not self.is_learner:
            for _ in range(self.cfg.actor_steps_per_learner_step):
                if not self.actor_step():
                    return False
            return True
        self._emu_push()
        self.learner_step()
        if self.transport == "p2p":
            self.ingest(self.ingest_cap)
        if self.learn_steps % self.cfg.publish_param_interval == 0:
            self.publish_params()
        self.links.check_heartbeats()
        return True

    @property
    def frames_per_actor_step(self) -> int:
        return self.E * 4
