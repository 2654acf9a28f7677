"""Greedy evaluator for the GPU engine (reference: origin_repo/eval.py:49-96).

The reference evaluator is one extra process: the latest published parameters, an
epsilon = 0 policy, ``clip_rewards`` forced off (episode returns in game points), the
same wrappers otherwise (episodic life on by default, ``max_episode_length`` 50000),
and ``evaluator/episode_reward`` / ``evaluator/episode_length`` logged per episode.

Here it is ``n_envs`` extra GPU envs with their own small frame ring (the training
replay's ring is never touched), their own copy of the network in the engine's
precision, and the same kernels as the actor shard: forward with the heads kernel's
action epilogue fed an all-zero epsilon (greedy), ``vec_env_step`` with reward
clipping off, and ``frame_hist_step`` advancing the observation stacks.  ``load`` copies
the latest published weights (the engine's actor weights, as the reference evaluator
takes the learner's PUB stream); ``run(k)`` advances every env ``k`` steps on the
caller's stream (a side stream in ``train.py``); ``poll()`` returns the episodes
finished since the last poll (a host read of the [E, 4] episode log).
"""
from __future__ import annotations

import torch

from .. import ops
from ..models.dqn import DuelingDQN
from .actor_shard import ENV_STATE_STRIDE
from .hbm_replay import FRAME_BYTES


class GPUEvaluator:
    def __init__(self, src_model: DuelingDQN, n_envs: int = 8, n_actions: int = 18, forward: str = "hip",
                 dtype: str = "fp32", device="cuda", seed: int = 0, episode_life: bool = True,
                 max_episode_steps: int = 50000, action_repeat: int = 4, epsilon: float = 0.0):
        self.hip = ops.hip()
        self.device = torch.device(device)
        self.E, self.A = int(n_envs), int(n_actions)
        self.seed = int(seed)
        E, dev = self.E, self.device
        self.model = DuelingDQN.from_shapes((4, 84, 84), self.A).to(dev)
        self.model.load_state_dict(src_model.state_dict())
        self.flat = self.model.flatten_parameters()
        for p in self.model.parameters():
            p.requires_grad_(False)
        self.forward_mode, self.dtype = forward, dtype
        if forward == "hip":
            from ..models.fused import make_hip_net, make_workspace

            self.net = make_hip_net(self.model, dtype)
            self.ws = make_workspace(E, self.A, dev, dtype)
        # frames live (2 x 4) steps in the ring: the stack needs the last 4
        self.F = E * 8
        self.frames = torch.zeros(self.F, FRAME_BYTES, dtype=torch.uint8, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.env_state = torch.zeros(E, ENV_STATE_STRIDE, **f32)
        self.new_frame = torch.zeros(E, **i32)
        self.hist = torch.zeros(E, 4, **i32)
        self.ep_log = torch.zeros(E, 4, **f32)
        self.reward = torch.zeros(E, **f32)
        self.done = torch.zeros(E, **f32)
        self.actions = torch.zeros(E, **i32)
        # greedy (reference: model.act(state, 0.)); epsilon 1 = the uniform-random baseline
        self.eps = torch.full((E,), float(epsilon), **f32)
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.obs = torch.zeros(E, 4, 84, 84, dtype=torch.uint8, device=dev)
        self.params = self.hip.VecEnvParams(E, self.A, FRAME_BYTES, self.F, action_repeat, 0, int(episode_life),
                                            int(max_episode_steps))
        self.hip.vec_env_reset(self.env_state.data_ptr(), self.seed, self.frames.data_ptr(), self.params,
                               self.counter.data_ptr(), self.new_frame.data_ptr(), self.hist.data_ptr(),
                               self.ep_log.data_ptr(), self._stream())
        self._seen = torch.zeros(E)
        self.episodes = 0
        self.steps = 0
        self.max_episode_steps = int(max_episode_steps)
        self._graph, self._graph_steps = None, 0

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def load(self, flat: torch.Tensor, net=None) -> None:
        """Take the latest published weights (flat fp32 buffer of the same architecture;
        ``net``: the source's HIP net, whose packed copies are copied instead of re-derived)."""
        self.hip.copy_f32(self.flat.data_ptr(), flat.data_ptr(), self.flat.numel(), self._stream())
        if self.forward_mode == "hip":
            if net is not None and type(net) is type(self.net):
                self.net.copy_packed_from(net)
            else:
                self.net.repack()

    def step(self) -> None:
        """One greedy step of every evaluator env."""
        h, s = self.hip, self._stream()
        if self.forward_mode == "hip":
            self.net(self.frames, self.ws, self.hist,
                     act=(self.eps.data_ptr(), self.seed ^ 0xE7A1, self.counter.data_ptr(), self.actions.data_ptr()))
        else:
            from .learner import forward_q

            self.hip.gather_frames(self.frames.data_ptr(), FRAME_BYTES, self.hist.data_ptr(), self.E, 4,
                                   self.obs.data_ptr(), s)
            with torch.no_grad():
                q = forward_q(self.model, self.obs, self.dtype == "bf16")
            self.hip.select_actions(q.contiguous().data_ptr(), self.E, self.A, self.eps.data_ptr(), self.seed ^ 0xE7A1,
                                    self.counter.data_ptr(), self.actions.data_ptr(), s)
        h.vec_env_step(self.env_state.data_ptr(), self.actions.data_ptr(), self.seed, self.counter.data_ptr(),
                       self.frames.data_ptr(), self.params, self.reward.data_ptr(), self.done.data_ptr(),
                       self.new_frame.data_ptr(), self.ep_log.data_ptr(), s)
        h.frame_hist_step(self.hist.data_ptr(), self.new_frame.data_ptr(), self.done.data_ptr(), self.E,
                          self.counter.data_ptr(), s)
        self.steps += 1

    def run(self, n_steps: int) -> None:
        """``n_steps`` greedy steps of every env: whole replays of the captured chunk graph
        (:meth:`capture`) while they fit, eager steps for the rest."""
        if self._graph is not None:
            for _ in range(n_steps // self._graph_steps):
                self._graph.replay()
                self.steps += self._graph_steps
            n_steps %= self._graph_steps
        for _ in range(n_steps):
            self.step()

    def capture(self, steps: int = 100) -> None:
        """Capture ``steps`` greedy steps as one hipGraph on the current stream (the
        evaluator's ~8 launches per step are host-bound when eager: a budget that finishes
        capped episodes is thousands of steps per log window)."""
        self.step()  # (a real step: every kernel's first launch happens outside the capture)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(steps):
                self.step()
        self.steps -= steps  # the captured steps did not run
        self._graph, self._graph_steps = g, int(steps)

    def running(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(return so far, steps so far) of every env's episode in progress (one host read):
        the explicit marker for episodes still running at a log line."""
        st = self.env_state[:, 25:27].cpu()  # S_EPRET, S_EPLEN (actor_kernels.hip)
        return st[:, 0], st[:, 1]

    def poll(self) -> list[tuple[float, float]]:
        """(episode_reward, episode_length) of the episodes finished since the last poll
        (the last one per env if an env finished several: the log keeps one per env)."""
        log = self.ep_log.cpu()
        out = []
        for e in range(self.E):
            if log[e, 2] > self._seen[e]:
                out.append((float(log[e, 0]), float(log[e, 1])))
        self.episodes += int((log[:, 2] - self._seen).clamp_min(0).sum())
        self._seen = log[:, 2].clone()
        return out
