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
all-gathered before the learner graph).
"""
from __future__ import annotations

import copy
import time
from dataclasses import dataclass, field

import torch

from ..models.dqn import DuelingDQN
from ..models.fused import HipDuelingNet, NetWorkspace
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
    exact_mass: bool = True
    seed: int = 1122
    learner: LearnerConfig = field(default_factory=LearnerConfig)


class ApexEngine:
    def __init__(self, cfg: EngineConfig, device: str | torch.device = "cuda", allreduce=None,
                 model: DuelingDQN | None = None, sharded: bool = False):
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

            self._sharded = ShardedSampling(self.replay)
        self.learner = DQNLearner(model, self.replay, lc, allreduce=allreduce, sharded=self._sharded)
        self.actor_model = copy.deepcopy(self.learner.model)
        self.actor_model._flat = None
        self.actor_flat = self.actor_model.flatten_parameters()
        for p in self.actor_model.parameters():
            p.requires_grad_(False)
            p.grad = None
        self.hip_net = lc.forward == "hip"
        if self.hip_net:
            self.actor_net = HipDuelingNet(self.actor_model)
            self.actor_ws = NetWorkspace(cfg.n_envs, cfg.n_actions, self.device)
        self.publish_params()
        self.learn_steps = 0
        self.actor_steps = 0
        self._g_actor = self._g_learn_a = self._g_learn_b = None
        self._pool = None
        self._captured = False
        self._allreduce = allreduce
        # overlap: staging half h (sets h*k .. h*k+k-1) is filled by the actor steps of one
        # train step while the learner applies the other half (the previous step's)
        self._half = 0
        self._astream = torch.cuda.Stream(device=self.device) if self.overlap else None
        self._ev_actor = [torch.cuda.Event(), torch.cuda.Event()] if self.overlap else None
        self._ev_learn = torch.cuda.Event() if self.overlap else None

    # ------------------------------------------------------------------ eager bodies
    def publish_params(self) -> None:
        """Learner -> local actor weights (the on-GPU analogue of learner.py:169-170)."""
        self.learner.copy_params_to(self.actor_flat)
        if self.hip_net:
            self.actor_net.copy_packed_from(self.learner.net)

    def _actor_body(self, stage: int | None = None):
        if self.hip_net:  # conv1 reads the current stacks straight from the frame ring
            q = self.actor_net(self.replay.frames, self.actor_ws, self.actor.st["hist"])
        else:
            obs = self.actor.observe()
            with torch.no_grad():
                q = forward_q(self.actor_model, obs)
        self.actor.act_and_step(q, stage)

    def _actor_half(self, half: int):
        k = self.cfg.actor_steps_per_learner_step
        for i in range(k):
            self._actor_body(half * k + i)

    def _apply_half(self, half: int):
        k = self.cfg.actor_steps_per_learner_step
        for i in range(k):
            self.actor.apply_staged(half * k + i)

    def _learn_a(self, apply_half: int | None = None):
        if apply_half is not None and self._sharded is None:
            # rows now (before sampling: a sampled slot never changes under the learner);
            # their priorities on the learner's tree stream, beside the backward (the new
            # transitions become sampleable one learner step later).  Sharded: applied in
            # full before the shard-mass exchange instead.
            k = self.cfg.actor_steps_per_learner_step
            for i in range(k):
                self.actor.apply_rows(apply_half * k + i)
            self.learner.tree_hooks = [lambda i=i: self.actor.apply_prios(apply_half * k + i) for i in range(k)]
        self.learner.sample_and_forward()

    def _learn_b(self):
        self.learner.optimize()

    # ------------------------------------------------------------------ graphs
    def capture(self, warmup_iters: int = 3) -> None:
        """Warm up on a side stream, then capture actor and learner steps as hipGraphs.
        The warm-up iterations are real train steps and are counted as such."""
        self.learn_steps += warmup_iters
        self.actor_steps += warmup_iters * self.cfg.actor_steps_per_learner_step
        if self.overlap:
            return self._capture_overlap(warmup_iters)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup_iters):
                self._actor_body()
                if self._sharded is not None:
                    self._sharded.exchange()
                self._learn_a()
                if self._allreduce is not None:
                    self._allreduce(self.learner.flat_grad)
                self._learn_b()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._pool = torch.cuda.graph_pool_handle()
        self._g_actor = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_actor, pool=self._pool):
            self._actor_body()
        self._g_learn_a = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_learn_a, pool=self._pool):
            self._learn_a()
            if self._allreduce is None:  # no host collective in between: one graph per step
                self._learn_b()
        self._g_learn_b = self._capture_learn_b()
        self._captured = True
        torch.cuda.synchronize(self.device)

    def _capture_learn_b(self):
        """The optimizer graph, needed only when an eager RCCL all-reduce sits between the
        backward and the optimizer (data-parallel); otherwise it is part of learn_a (each
        graph boundary costs ~8 us of launch gap, rocprofv3 trace)."""
        if self._allreduce is None:
            return None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self._pool):
            self._learn_b()
        return g

    def _capture_overlap(self, warmup_iters: int) -> None:
        """Overlap mode: graphs per staging half (actor: fill half h; learner: apply half
        1-h, sample, forward, backward) + the optimizer graph.  Warm-up runs real
        sequential train steps, keeping the one-step-behind staging invariant."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup_iters):
                self._train_step_eager()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._pool = torch.cuda.graph_pool_handle()
        apool = torch.cuda.graph_pool_handle()  # actor graphs run concurrently: never share memory
        self._g_actor, self._g_learn_a, self._g_apply = [], [], []
        for h in (0, 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=apool):
                self._actor_half(h)
            self._g_actor.append(g)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._pool):
                self._learn_a(1 - h)
                if self._allreduce is None:
                    self._learn_b()
            self._g_learn_a.append(g)
            if self._sharded is not None:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._pool):
                    self._apply_half(1 - h)
                self._g_apply.append(g)
        self._g_learn_b = self._capture_learn_b()
        self._captured = True
        torch.cuda.synchronize(self.device)
        self._ev_learn.record(torch.cuda.current_stream(self.device))

    def _train_step_eager(self) -> None:
        """Overlap-mode semantics, run sequentially on the current stream."""
        h = self._half
        self._actor_half(h)
        if self._sharded is not None:
            self._apply_half(1 - h)
            self._sharded.exchange()
        self._learn_a(1 - h)
        if self._allreduce is not None:
            self._allreduce(self.learner.flat_grad)
        self._learn_b()
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
        A.wait_event(self._ev_learn)
        with torch.cuda.stream(A):
            self._g_actor[h].replay()
        self._ev_actor[h].record(A)
        L.wait_event(self._ev_actor[1 - h])
        if self._sharded is not None:
            self._g_apply[h].replay()
            self._sharded.exchange()
        self._g_learn_a[h].replay()
        if self._allreduce is not None:
            self._allreduce(self.learner.flat_grad)
            self._g_learn_b.replay()
        self.learn_steps += 1
        self.actor_steps += self.cfg.actor_steps_per_learner_step
        if self.learn_steps % self.cfg.publish_param_interval == 0:
            L.wait_event(self._ev_actor[h])  # the actor is not reading its weights
            self.publish_params()
        if self.learn_steps % self.cfg.target_update_interval == 0:
            self.learner.sync_target()
        self._ev_learn.record(L)
        self._half ^= 1

    # ------------------------------------------------------------------ steps
    def actor_step(self) -> None:
        if self._g_actor is not None:
            self._g_actor.replay()
        else:
            self._actor_body()
        self.actor_steps += 1

    def learner_step(self) -> None:
        if self._sharded is not None:  # 16 B/rank all-gather of shard masses (eager collective)
            self._sharded.exchange()
        if self._g_learn_a is not None:
            self._g_learn_a.replay()
            if self._allreduce is not None:
                self._allreduce(self.learner.flat_grad)
                self._g_learn_b.replay()
        else:
            self._learn_a()
            if self._allreduce is not None:
                self._allreduce(self.learner.flat_grad)
            self._learn_b()
        self.learn_steps += 1
        if self.learn_steps % self.cfg.publish_param_interval == 0:
            self.publish_params()
        if self.learn_steps % self.cfg.target_update_interval == 0:
            self.learner.sync_target()

    def fill(self, min_transitions: int | None = None) -> None:
        """Run actor steps until the replay holds ``threshold_size`` slots."""
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
            return
        for _ in range(steps):
            self.actor_step()

    def train_step(self) -> None:
        """One Ape-X step of this rank: one learner SGD step + its actor steps."""
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
