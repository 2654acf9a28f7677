"""Central-replay Ape-X topology across GPUs (BASELINE config 3).

Rank 0 is the learner and holds the one HBM replay (frame ring + transition table +
priority tree), split into one region per actor rank.  Ranks 1..W-1 are actor GPUs:
each runs an :class:`ActorShard` (E GPU envs, batched MFMA inference with the global
Ape-X epsilon ladder, on-device n-step) writing into a *local mirror* of its region,
and after every actor step pushes the step's E new frames + E transition rows to rank 0
(``parallel.experience``: 2 point-to-point messages, RCCL over xGMI).  Rank 0 scatters
them into the region and writes their priorities into the tree; the learner samples
the union.  Every ``publish_param_interval`` learner steps rank 0 broadcasts its flat
parameters to all actor ranks (RCCL broadcast, ``parallel.broadcast``).

The step is lock-step (``actor_steps_per_learner_step`` pushes per learner step), so the
message order on every link is fixed and no host polling is needed.  This is the
reference's replay-server topology (actor.py -> replay.py <- learner.py) with ZMQ +
pickle replaced by device-to-device messages; the data-parallel *sharded* topology
(``ApexEngine`` with ``sharded=True``) is the other multi-GPU layout.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..models.dqn import DuelingDQN
from ..models.fused import make_hip_net, make_workspace
from ..parallel.experience import ExperienceReceiver, ExperienceSender, Region, apply_packet, pack_meta
from .actor_shard import ActorShard
from .apex import EngineConfig
from .hbm_replay import FRAME_BYTES, HBMReplay
from .learner import DQNLearner


def region_geometry(cfg: EngineConfig, n_actor_ranks: int) -> tuple[int, int]:
    """(transition slots, frame slots) per actor-rank region; multiples of the env count."""
    E, n = cfg.n_envs, cfg.learner.n_step
    c = max(E, (cfg.replay_capacity // max(1, n_actor_ranks)) // E * E)
    f = c + -(-(2 * n + 8) * E // E) * E
    return c, f


class CentralApexEngine:
    def __init__(self, cfg: EngineConfig, device, rank: int | None = None, world: int | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        if self.world < 2:
            raise ValueError("the central topology needs >= 2 ranks (rank 0 learner, ranks 1.. actors)")
        self.R = self.world - 1
        lc = cfg.learner
        E = cfg.n_envs
        self.E = E
        self.C_r, self.F_r = region_geometry(cfg, self.R)
        torch.manual_seed(cfg.seed)
        model = DuelingDQN.from_shapes((4, 84, 84), cfg.n_actions)
        self.is_learner = self.rank == 0
        self.via_host = dist.get_backend() != "nccl"
        self.learn_steps = self.actor_steps = 0
        self.rounds = 0  # lock-step rounds (identical on every rank: drives the broadcast cadence)
        self._g_actor = self._g_learn = None
        if self.is_learner:
            self.replay = HBMReplay(self.C_r * self.R, E, lc.n_step, cfg.alpha, self.device,
                                    frame_capacity=self.F_r * self.R, exact_mass=cfg.exact_mass, seed=cfg.seed)
            self.learner = DQNLearner(model, self.replay, lc)
            self.flat = self.learner.flat
            self.regions = {r: Region((r - 1) * self.C_r, self.C_r, (r - 1) * self.F_r, self.F_r)
                            for r in range(1, self.world)}
            self.receiver = ExperienceReceiver(E, FRAME_BYTES, self.device, range(1, self.world))
            rp = self.replay
            self.tables = {"frames": rp.frames, "s_ids": rp.s_ids, "s2_ids": rp.s2_ids, "action": rp.action,
                           "reward": rp.reward, "done": rp.done}
        else:
            self.replay = HBMReplay(self.C_r, E, lc.n_step, cfg.alpha, self.device, frame_capacity=self.F_r,
                                    exact_mass=cfg.exact_mass, seed=cfg.seed + self.rank)
            self.actor = ActorShard(self.replay, E, cfg.n_actions, lc.n_step, lc.gamma, cfg.eps_base, cfg.eps_alpha,
                                    actor_offset=(self.rank - 1) * E, total_actors=self.R * E,
                                    seed=cfg.seed + 7919 * self.rank, mode=cfg.nstep_mode)
            model = model.to(self.device)
            self.flat = model.flatten_parameters()
            for p in model.parameters():
                p.requires_grad_(False)
            self.model = model
            self.net = make_hip_net(model, cfg.learner.dtype)
            self.ws = make_workspace(E, cfg.n_actions, self.device, cfg.learner.dtype)
            self.sender = ExperienceSender(E, FRAME_BYTES, self.device, dst=0)
            self.pkt_frames = torch.empty(E, FRAME_BYTES, dtype=torch.uint8, device=self.device)
        self.broadcast_params()
        if not self.is_learner:  # the reset frames are the first packet
            self._stage_packet(initial=True)
            self.sender.send(self.pkt_frames, self.sender.meta)
        else:
            self._ingest()

    # ------------------------------------------------------------------ params
    def broadcast_params(self) -> None:
        """Rank 0 -> all actor ranks (RCCL broadcast of the 3.5 MB flat buffer)."""
        if self.via_host:
            h = self.flat.cpu()
            dist.broadcast(h, src=0)
            if not self.is_learner:
                self.flat.copy_(h)
        else:
            dist.broadcast(self.flat, src=0)
        if not self.is_learner:
            self.net.repack()

    # ------------------------------------------------------------------ actor ranks
    def _stage_packet(self, initial: bool = False) -> None:
        a, rp = self.actor, self.replay
        if initial:  # reset frames only: no transition rows (priority 0)
            z = torch.zeros(self.E, dtype=torch.float32, device=self.device)
            slot = torch.arange(self.E, dtype=torch.int32, device=self.device)
            pack_meta(a.st["hist"], a.st["hist"], a.actions, z, z, z, slot, a.new_frame, out=self.sender.meta)
        else:
            sl = a.slot.long()
            pack_meta(rp.s_ids.index_select(0, sl), rp.s2_ids.index_select(0, sl), rp.action.index_select(0, sl),
                      rp.reward.index_select(0, sl), rp.done.index_select(0, sl), a.prio, a.slot, a.new_frame,
                      out=self.sender.meta)
        torch.index_select(rp.frames, 0, a.new_frame.long(), out=self.pkt_frames)

    def _actor_body(self) -> None:
        q = self.net(self.replay.frames, self.ws, self.actor.st["hist"])
        self.actor.act_and_step(q)
        self._stage_packet()

    def actor_step(self) -> None:
        self.sender.wait()  # the previous packet left the staging buffers
        if self._g_actor is not None:
            self._g_actor.replay()
        else:
            self._actor_body()
        self.sender.send(self.pkt_frames, self.sender.meta)
        self.actor_steps += 1

    # ------------------------------------------------------------------ learner rank
    def _ingest(self) -> None:
        self.receiver.post()
        slots, prios = [], []
        for r, (frames, meta) in self.receiver.take(self.device).items():
            sl, pr = apply_packet(self.tables, self.regions[r], frames, meta)
            slots.append(sl)
            prios.append(pr)
        self.replay.write_priorities(torch.cat(slots), torch.cat(prios), dedup=False,
                                     bumps=((self.replay.filled, self.E * self.R),))

    def learner_step(self) -> None:
        if self._g_learn is not None:
            self._g_learn.replay()
        else:
            self.learner.step()
        self.learn_steps += 1
        if self.learn_steps % self.cfg.target_update_interval == 0:
            self.learner.sync_target()

    # ------------------------------------------------------------------ lock-step driver
    def fill_steps(self) -> int:
        return max(4, -(-self.cfg.threshold_size // (self.E * self.R)))

    def fill(self) -> None:
        for _ in range(self.fill_steps()):
            if self.is_learner:
                self._ingest()
            else:
                self.actor_step()

    def _round_eager(self) -> None:
        if self.is_learner:
            self.learner.step()
            self.learn_steps += 1
            for _ in range(self.cfg.actor_steps_per_learner_step):
                self._ingest()
        else:
            for _ in range(self.cfg.actor_steps_per_learner_step):
                self.actor_step()

    def capture(self, warmup_rounds: int = 3) -> None:
        """Warm up with real lock-step rounds (messages included, so every link keeps
        its per-round message count), then capture the compute-only bodies; the
        messages stay eager around the graph replays."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup_rounds):
                self._round_eager()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        pool = torch.cuda.graph_pool_handle()
        if self.is_learner:
            self._g_learn = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_learn, pool=pool, capture_error_mode="thread_local"):
                self.learner.step()
        else:
            self.sender.wait()
            self._g_actor = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_actor, pool=pool, capture_error_mode="thread_local"):
                self._actor_body()
        torch.cuda.synchronize(self.device)

    def train_step(self) -> None:
        """One lock-step round: rank 0 = 1 learner step + ingest of every actor rank's
        pushes; actor ranks = ``actor_steps_per_learner_step`` actor steps + pushes."""
        k = self.cfg.actor_steps_per_learner_step
        if self.is_learner:
            self.learner_step()
            for _ in range(k):
                self._ingest()
        else:
            for _ in range(k):
                self.actor_step()
        self.rounds += 1
        if self.rounds % self.cfg.publish_param_interval == 0:
            if not self.is_learner:
                self.sender.wait()
            self.broadcast_params()

    @property
    def frames_per_actor_step(self) -> int:
        return self.E * 4
