"""Single-GPU (per rank) Ape-X engine: actor shard + HBM replay + fused learner.

This is the MI355X-native replacement for the reference's three process kinds
(actor / replay server / learner talking ZeroMQ + pickle) on one GPU:

* actor shard: ``n_envs`` GPU envs with the global epsilon ladder (ActorShard)
* replay: HBM frame ring + fanout-64 priority tree (HBMReplay)
* learner: fused double-DQN step (DQNLearner)

Each is a static sequence of kernels captured once into a hipGraph (via
``torch.cuda.CUDAGraph``) and replayed; the host only replays graphs and counts
steps.  Reference cadences are kept: params published to the actors every
``publish_param_interval`` learner steps (learner.py:169, 25), target sync every
``target_update_interval`` (learner.py:163, 2500), learning starts after
``threshold_size`` transitions (replay.py:104, 50,000).  In data-parallel mode (one
rank per GPU, ``apex_amd.parallel``), the flat gradient is all-reduced over RCCL
between the two learner graphs, and with ``sharded=True`` the replay shards are
sampled as one global prioritized buffer (``parallel.sharded``: shard masses are
all-gathered before the learner graph).  The data-parallel step is split into three
phase graphs so the FC1/head gradient all-reduce overlaps the conv backward
(``ApexEngine._learn``).
"""
from __future__ import annotations

import copy
import time
from dataclasses import dataclass, field

import torch

from .. import ops
from ..models.dqn import DuelingDQN
from ..utils import trace
from ..models.fused import make_hip_net, make_workspace
from .actor_shard import ActorShard
from .hbm_replay import HBMReplay
from .learner import DQNLearner, LearnerConfig, forward_q



@dataclass
class EngineConfig:
    n_envs: int = 256                    # actors (envs) on this GPU
    n_actions: int = 18                  # Seaquest (the reference's published run)
    replay_capacity: int = 2_000_000     # arguments.py --replay_buffer_size
    alpha: float = 0.6
    threshold_size: int = 50_000
    actor_steps_per_learner_step: int = 1
    publish_param_interval: int = 25
    target_update_interval: int = 2500
    nstep_mode: str = "reference"
    eps_base: float = 0.4
    eps_alpha: float = 7.0
    actor_offset: int = 0
    total_actors: int | None = None
    use_graphs: bool = True
    overlap: bool = False                # actor graph on its own stream, concurrent with the learner
    exact_mass: bool = False             # SURVEY Q5 parity: the newest slot is excluded from the sampled mass
    # data-parallel overlap mode: capture the whole learner step INCLUDING the two RCCL
    # gradient all-reduces (direct communicator, parallel/rccl.py) as one hipGraph per
    # staging half, instead of three phase graphs with eager collectives in between
    dp_graph: bool = False
    # overlap mode, single process: where the actor graph starts within the learner step --
    # "start" (with the step) or "loss" (after the fused loss + heads backward: the actor's
    # forward then co-runs with the trunk backward and the optimizer instead of the
    # learner's forward GEMMs; the learner graph is split there, one launch boundary)
    actor_at: str = "start"
    seed: int = 1122
    learner: LearnerConfig = field(default_factory=LearnerConfig)


_RESERVED: dict = {}


def reserve_actor_stream(device) -> None:
    """Take the actor's stream from torch's stream pool NOW -- call it before
    ``init_process_group`` and anything else that draws pool streams.  Pool streams are
    spread round-robin over the GPU's hardware queues (GPU_MAX_HW_QUEUES = 4); the
    process group's RCCL stream drawn first shifts the actor's stream onto the learner's
    queue (rocprofv3: actor and learner kernels strictly interleaved on one queue, 0.51
    vs 0.31 ms/step).  Reserving first gives every rank the single-process layout."""
    dev = torch.device(device)
    if dev not in _RESERVED:
        _RESERVED[dev] = torch.cuda.Stream(device=dev)


class ApexEngine:
    def __init__(self, cfg: EngineConfig, device: str | torch.device = "cuda", allreduce=None,
                 model: DuelingDQN | None = None, sharded: bool = False, force_collectives: bool = False):
        """``allreduce``: data-parallel gradient all-reduce (``parallel.dp.FlatGradAllReduce``
        over torch.distributed, or ``parallel.rccl.RcclGradAllReduce``, direct RCCL); the
        shard-mass exchange uses the same object."""
        self.cfg = cfg
        self.device = torch.device(device)
        lc = cfg.learner
        torch.manual_seed(cfg.seed)
        self.replay = HBMReplay(cfg.replay_capacity, cfg.n_envs, lc.n_step, cfg.alpha, self.device,
                                exact_mass=cfg.exact_mass, seed=cfg.seed)
        k = cfg.actor_steps_per_learner_step
        self.overlap = bool(cfg.overlap)
        self.actor = ActorShard(self.replay, cfg.n_envs, cfg.n_actions, lc.n_step, lc.gamma, cfg.eps_base,
                                cfg.eps_alpha, cfg.actor_offset, cfg.total_actors, cfg.seed, cfg.nstep_mode,
                                staged=2 * k if self.overlap else 0)
        model = model if model is not None else DuelingDQN.from_shapes((4, 84, 84), cfg.n_actions)
        self._sharded = None
        if sharded:
            from ..parallel.sharded import ShardedSampling

            self._sharded = ShardedSampling(self.replay, force=force_collectives, comm=allreduce)
        self.learner = DQNLearner(model, self.replay, lc, allreduce=allreduce, sharded=self._sharded)
        self.actor_model = copy.deepcopy(self.learner.model)
        self.actor_model._flat = None
        self.actor_flat = self.actor_model.flatten_parameters()
        for p in self.actor_model.parameters():
            p.requires_grad_(False)
            p.grad = None
        self.hip_net = lc.forward == "hip"
        if self.hip_net:
            # actors act at the learner's precision (the reference's actors are fp32 too)
            self.actor_net = make_hip_net(self.actor_model, lc.dtype)
            self.actor_ws = make_workspace(cfg.n_envs, cfg.n_actions, self.device, lc.dtype)
            self.actor_ws.q = self.actor.q  # the heads kernel writes the actor's Q in place (no copy)
        self.publish_params()
        self.learn_steps = 0
        self.actor_steps = 0
        self._g_actor = self._g_learn_a = self._g_learn_a2 = self._g_learn_b = self._g_dp = None
        self._pool = None
        self._mass_pending = False  # next step's shard masses already exchanged (with the conv grads)
        self._captured = False
        self._allreduce = allreduce
        # overlap: staging half h (sets h*k .. h*k+k-1) is filled by the actor steps of one
        # train step while the learner applies the other half (the previous step's)
        self._half = 0
        # the actor stream: the one reserve_actor_stream took before the process group drew
        # its pool streams, else the next pool stream
        self._astream = (_RESERVED.pop(self.device, None) or torch.cuda.Stream(device=self.device)) if self.overlap \
            else None
        self._ev_actor = [torch.cuda.Event(), torch.cuda.Event()] if self.overlap else None
        self._ev_learn = torch.cuda.Event() if self.overlap else None
        if cfg.actor_at not in ("start", "loss"):
            raise ValueError("EngineConfig.actor_at must be 'start' or 'loss'")
        # the learner graph split at the loss (the actor launches between its two halves)
        self._split_at_loss = (self.overlap and cfg.actor_at == "loss" and self.hip_net and allreduce is None
                               and not lc.private_rows)
        self._g_learn_front = None

    # ------------------------------------------------------------------ eager bodies
    def publish_params(self) -> None:
        """Learner -> local actor weights (the on-GPU analogue of learner.py:169-170)."""
        trace.mark("apex.publish_params")
        self.learner.copy_params_to(self.actor_flat)
        if self.hip_net:
            self.actor_net.copy_packed_from(self.learner.net)

    def _actor_body(self, stage: int | None = None):
        if self.hip_net:  # conv1 reads the current stacks straight from the frame ring; the
            # heads kernel writes Q into the actor's buffer and picks the eps-greedy actions
            self.actor_net(self.replay.frames, self.actor_ws, self.actor.st["hist"], act=self.actor.act_args())
            self.actor.act_and_step(None, stage, selected=True)
            return
        else:
            obs = self.actor.observe()
            with torch.no_grad():
                q = forward_q(self.actor_model, obs, self.cfg.learner.dtype == "bf16")
        self.actor.act_and_step(q, stage)

    def _actor_half(self, half: int):
        """Actor steps into staging half ``half``."""
        k = self.cfg.actor_steps_per_learner_step
        for i in range(k):
            self._actor_body(half * k + i)

    def _apply_half(self, half: int):
        k = self.cfg.actor_steps_per_learner_step
        for i in range(k):
            self.actor.apply_staged(half * k + i)

    def _learn_a(self, apply_half: int | None = None):
        """Overlap mode: apply the staged actor rows of ``apply_half`` (before sampling: a
        sampled slot never changes under the learner) and defer their priorities to the
        learner's tree stream, beside the backward (the new transitions become sampleable
        one learner step later -- which also keeps a sharded rank's exchanged shard mass
        equal to the tree it samples).  Then the forward phase (single-process: the whole
        learner step up to the optimizer)."""
        if apply_half is not None:
            k = self.cfg.actor_steps_per_learner_step
            if self.hip_net:  # rows scattered by the sampling launch itself
                self.learner.pre_rows = [self.actor.staged_rows(apply_half * k + i) for i in range(k)]
            else:
                for i in range(k):
                    self.actor.apply_rows(apply_half * k + i)
            self.learner.pre_writes = [self.actor.staged_prio_write(apply_half * k + i) for i in range(k)]
        self.learner.forward_phase()

    def _learn_front(self, apply_half: int) -> None:
        """Split-at-loss learner graph, first half: staged actor rows + sample + forward x3 +
        the fused loss / heads backward."""
        self._stage_rows(apply_half)
        self.learner.forward_phase(part="a")

    def _stage_rows(self, apply_half: int) -> None:
        k = self.cfg.actor_steps_per_learner_step
        self.learner.pre_rows = [self.actor.staged_rows(apply_half * k + i) for i in range(k)]
        self.learner.pre_writes = [self.actor.staged_prio_write(apply_half * k + i) for i in range(k)]

    def _learn_b(self):
        self.learner.optimize()

    @property
    def _dp(self) -> bool:
        return self._allreduce is not None and self.learner.dp_split

    def _learn(self, a1, a2, b, pipelined_mass: bool) -> None:
        """One learner step from its phases (graph replays or eager bodies).

        Data-parallel (one rank per GPU, RCCL over xGMI)::

            [wait shard-mass all-gather] a1 | start all-reduce(FC1+heads grads) | a2 (conv
            backward) | start all-reduce(conv grads) [| start next step's mass all-gather]
            | wait both | b (optimizer, 1/world mean folded in)

        The FC1/head slice (~3.2 of 3.5 MB) travels while the conv backward computes; the
        mass all-gather of step t+1 travels while the optimizer of step t runs
        (``pipelined_mass``: only when no actor writes the tree between steps, i.e. in
        overlap mode where actor rows are staged and applied by the learner).
        Single-process: ``a1`` is the whole step and ``a2``/``b`` are None."""
        with trace.range("apex.learner"):
            self._learn_phases(a1, a2, b, pipelined_mass)

    def _learn_phases(self, a1, a2, b, pipelined_mass: bool) -> None:
        R = trace.range
        sh = self._sharded
        if sh is not None and not self._mass_pending:
            with R("mass.exchange"):
                sh.exchange()
        self._mass_pending = False
        with R("learn.a1"):
            a1()
        if a2 is None:
            return
        ar = self._allreduce
        fc, conv = self.learner.grad_slices()
        with R("ar.fc.start"):
            w1 = ar.start(fc)
        with R("learn.a2"):
            a2()  # (sharded: ends by packing this shard's slot in front of the conv grads)
        with R("ar.conv.start"):
            w2 = ar.start(conv)
        # the slots travelled with the conv grads: the next step's masses are exchanged
        # (valid when no actor writes the tree in between: overlap mode)
        self._mass_pending = sh is not None and pipelined_mass and self.learner.grad_prefix > 0
        with R("ar.wait"):
            ar.wait(w1, w2)
        with R("learn.b"):
            b()

    def _drain_mass(self) -> None:
        """Something other than a train step is about to touch the tree: the pipelined
        shard masses are stale, re-exchange at the next step."""
        self._mass_pending = False

    # ------------------------------------------------------------------ graphs
    @staticmethod
    def _graph(fn, pool):
        # thread_local capture: the process group's watchdog thread polls RCCL work events
        # while we capture; in the default (global) mode that call invalidates the capture
        # ("operation not permitted when stream is capturing", seen with --force-dp)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
            fn()
        return g

    def capture(self, warmup_iters: int = 3, warm_replays: int = 0) -> None:
        """Warm up on a side stream, then capture actor and learner steps as hipGraphs.
        The warm-up iterations are real train steps and are counted as such.  Collectives
        stay eager, between the learner's phase graphs (unless ``dp_graph``).
        ``warm_replays``: real train steps through the captured graphs right after capture,
        back to back (also counted): after a pause the MI355X runs the first ~30 steps 4-8 %
        slower than steady state (clock / power ramp, scripts/diag/warmup_curve.py), so a
        caller that times a short window right after setup starts from the sustained state."""
        self._drain_mass()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup_iters):  # full eager train steps (counters, publish/target cadence)
                self.train_step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._pool = torch.cuda.graph_pool_handle()
        if self.overlap:
            self._capture_overlap_graphs(torch.cuda.graph_pool_handle())  # actor graphs run concurrently:
        else:                                                           # never share their memory
            L = self.learner
            self._g_actor = self._graph(self._actor_body, self._pool)
            if self._dp:
                self._g_learn_a = self._graph(L.forward_phase, self._pool)
                self._g_learn_a2 = self._graph(L.backward_phase, self._pool)
                self._g_learn_b = self._graph(self._learn_b, self._pool)
            else:  # no host collective in between: one graph per step
                self._g_learn_a = self._graph(lambda: (L.forward_phase(), self._learn_b()), self._pool)
        self._captured = True
        torch.cuda.synchronize(self.device)
        if self.overlap:
            self._ev_learn.record(torch.cuda.current_stream(self.device))
        for _ in range(warm_replays):
            self.train_step()

    def _capture_overlap_graphs(self, apool) -> None:
        """Overlap mode: graphs per staging half (actor: fill half h; learner: apply half
        1-h, sample, forward, backward [, optimizer]); data-parallel: the learner's three
        phase graphs per half, or ONE graph per half with the all-reduces inside."""
        self._g_actor, self._g_learn_a, self._g_learn_a2 = [], [], []
        self._g_dp = None
        if self._dp and self.cfg.dp_graph and self._mass_pending_ok():
            # the whole data-parallel learner step -- both gradient all-reduces included
            # (RCCL kernels on the comm stream's branch of the graph) -- as ONE graph per half
            try:
                g_actor, g_dp = [], []
                for h in (0, 1):
                    g_actor.append(self._graph(lambda h=h: self._actor_half(h), apool))
                    g_dp.append(self._graph(lambda h=h: self._dp_step_body(1 - h), self._pool))
                self._g_actor, self._g_dp = g_actor, g_dp
                return
            except RuntimeError as e:  # RCCL capture unsupported here: the phase graphs instead
                import warnings

                warnings.warn(f"capturing the RCCL all-reduces failed ({e}); using three phase graphs")
                self._g_dp = None
                torch.cuda.synchronize(self.device)
                apool = torch.cuda.graph_pool_handle()
        if self._split_at_loss:
            L = self.learner
            self._g_learn_front = []
            for h in (0, 1):
                self._g_actor.append(self._graph(lambda h=h: self._actor_half(h), apool))
                self._g_learn_front.append(self._graph(lambda h=h: self._learn_front(1 - h), self._pool))
                self._g_learn_a.append(self._graph(lambda: (L.forward_phase(part="b"), self._learn_b()), self._pool))
            self._g_learn_b = None
            return
        for h in (0, 1):
            self._g_actor.append(self._graph(lambda h=h: self._actor_half(h), apool))
            if self._dp:
                self._g_learn_a.append(self._graph(lambda h=h: self._learn_a(1 - h), self._pool))
                self._g_learn_a2.append(self._graph(self.learner.backward_phase, self._pool))
            else:
                self._g_learn_a.append(self._graph(lambda h=h: (self._learn_a(1 - h), self._learn_b()), self._pool))
        self._g_learn_b = self._graph(self._learn_b, self._pool) if self._dp else None

    def _mass_pending_ok(self) -> bool:
        """One-graph DP step: the shard masses must always arrive with the previous step's
        conv-gradient all-reduce (overlap mode, slots in the gradient prefix)."""
        return self._sharded is None or (self.overlap and self.learner.grad_prefix > 0)

    def _dp_step_body(self, apply_half: int) -> None:
        """Captured body of the one-graph DP step (EngineConfig.dp_graph)."""
        ar = self._allreduce
        self._learn_a(apply_half)
        fc, conv = self.learner.grad_slices()
        # the FC1/head all-reduce depends on this point but is captured after the conv
        # backward's first launch, so the backward chain keeps the graph's queue
        ready, w = ar.mark(), []
        self.learner.backward_phase(after_first=lambda: w.append(ar.start(fc, ready=ready)))
        w1 = w[0]
        w2 = ar.start(conv)
        ar.wait(w1, w2)
        self._learn_b()

    def _learner_eager(self, apply_half: int | None = None) -> None:
        if self._dp:
            self._learn(lambda: self._learn_a(apply_half), self.learner.backward_phase, self._learn_b, False)
        else:
            self._learn(lambda: (self._learn_a(apply_half), self._learn_b()), None, None, False)

    def _train_step_eager(self) -> None:
        """Overlap-mode semantics, run sequentially on the current stream."""
        h = self._half
        self._actor_half(h)
        self._learner_eager(1 - h)
        self._half ^= 1

    def _train_step_overlap(self) -> None:
        """Actor half h on the actor stream || learner step on the current stream.

        Ordering (events): actor step t waits for learner step t-1 (which applied the
        staging half this actor step refills, and published weights); learner step t
        waits for actor step t-1 (whose half it applies).  The frame ring's margin
        ((2n+8)E frames beyond the transition capacity) keeps every frame the actor
        overwrites unreferenced by any sampleable transition."""
        h = self._half
        L = torch.cuda.current_stream(self.device)
        A = self._astream
        if self._g_learn_front is not None:
            self._train_step_split(h, L, A)
            return
        with trace.range("actor.launch"):
            A.wait_event(self._ev_learn)
            with torch.cuda.stream(A):
                self._g_actor[h].replay()
            self._ev_actor[h].record(A)
            L.wait_event(self._ev_actor[1 - h])
        if self._g_dp is not None:
            if self._sharded is not None and not self._mass_pending:  # e.g. after fill(): re-exchange
                self._sharded.exchange()
            with trace.range("apex.learner"):
                self._g_dp[h].replay()
            self._mass_pending = self._sharded is not None  # the graph's conv all-reduce carried them
        elif self._dp:
            self._learn(self._g_learn_a[h].replay, self._g_learn_a2[h].replay, self._g_learn_b.replay, True)
        else:
            self._learn(self._g_learn_a[h].replay, None, None, False)
        self.learn_steps += 1
        self.actor_steps += self.cfg.actor_steps_per_learner_step
        if self.learn_steps % self.cfg.publish_param_interval == 0:
            L.wait_event(self._ev_actor[h])  # the actor is not reading its weights
            self.publish_params()
        if self.learn_steps % self.cfg.target_update_interval == 0:
            self.learner.sync_target()
        self._ev_learn.record(L)
        self._half ^= 1

    def _train_step_split(self, h: int, L, A) -> None:
        """actor_at="loss": learner front (sample .. loss + heads backward) | actor half h on
        the actor stream from there, beside the learner's trunk backward + optimizer.  Same
        ordering as :meth:`_train_step_overlap`: actor step t follows learner step t-1 (L is in
        order, the front of step t comes after it) and learner step t waits for actor t-1."""
        with trace.range("apex.learner"):
            L.wait_event(self._ev_actor[1 - h])
            self._g_learn_front[h].replay()
        with trace.range("actor.launch"):
            self._ev_learn.record(L)
            A.wait_event(self._ev_learn)
            with torch.cuda.stream(A):
                self._g_actor[h].replay()
            self._ev_actor[h].record(A)
        with trace.range("apex.learner"):
            self._g_learn_a[h].replay()
        self.learn_steps += 1
        self.actor_steps += self.cfg.actor_steps_per_learner_step
        if self.learn_steps % self.cfg.publish_param_interval == 0:
            L.wait_event(self._ev_actor[h])  # the actor is not reading its weights
            self.publish_params()
        if self.learn_steps % self.cfg.target_update_interval == 0:
            self.learner.sync_target()
        self._half ^= 1

    # ------------------------------------------------------------------ steps
    def actor_step(self) -> None:
        self._drain_mass()
        if self._g_actor is not None:
            self._g_actor.replay()
        else:
            self._actor_body()
        self.actor_steps += 1

    def learner_step(self) -> None:
        if self._g_learn_a is None:
            self._learner_eager()
        elif self._dp:
            self._learn(self._g_learn_a.replay, self._g_learn_a2.replay, self._g_learn_b.replay, False)
        else:
            self._learn(self._g_learn_a.replay, None, None, False)
        self.learn_steps += 1
        if self.learn_steps % self.cfg.publish_param_interval == 0:
            self.publish_params()
        if self.learn_steps % self.cfg.target_update_interval == 0:
            self.learner.sync_target()

    def fill(self, min_transitions: int | None = None) -> None:
        """Run actor steps until the replay holds ``threshold_size`` slots."""
        self._drain_mass()
        need = self.cfg.threshold_size if min_transitions is None else min_transitions
        steps = max(-(-need // self.cfg.n_envs), 4)
        if self.overlap:  # whole halves; the last one stays staged for the first learner step
            k = self.cfg.actor_steps_per_learner_step
            halves = max(2, -(-steps // k))
            for i in range(halves):
                self._actor_half(self._half)
                if i < halves - 1:
                    self._apply_half(self._half)
                self._half ^= 1
                self.actor_steps += k
        else:
            for _ in range(steps):
                self.actor_step()

    def train_step(self) -> None:
        """One Ape-X step of this rank: one learner SGD step + its actor steps."""
        if trace.enabled():
            with trace.range("apex.train_step"):
                return self._train_step()
        return self._train_step()

    def _train_step(self) -> None:
        if self.overlap:
            if self._captured:
                self._train_step_overlap()
            else:
                self._train_step_eager()
                self.learn_steps += 1
                self.actor_steps += self.cfg.actor_steps_per_learner_step
                if self.learn_steps % self.cfg.publish_param_interval == 0:
                    self.publish_params()
                if self.learn_steps % self.cfg.target_update_interval == 0:
                    self.learner.sync_target()
            return
        self.learner_step()
        for _ in range(self.cfg.actor_steps_per_learner_step):
            self.actor_step()

    def run(self, n_steps: int) -> float:
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        for _ in range(n_steps):
            self.train_step()
        torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0

    @property
    def frames_per_actor_step(self) -> int:
        return self.cfg.n_envs * 4  # action repeat 4 (MaxAndSkipEnv)

    def save(self, path: str) -> None:
        torch.save(self.learner.model.state_dict(), path)
