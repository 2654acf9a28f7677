"""GPU actor shard: E vectorised envs + batched inference + on-device n-step batcher.

Replaces the reference's per-process actor loop (origin_repo/actor.py:52-115,
batchrecorder.py:42-78): one actor step of the whole shard is

  gather obs stacks (frame ids -> u8 [E,4,84,84])  ->  Q = policy(obs) [E,A]
  -> epsilon-greedy with the Ape-X ladder eps_i = 0.4^(1 + 7 i/(N-1)) on device
  -> vec env step (renders new frames straight into the HBM frame ring)
  -> n-step emit (transition + actor-computed priority written into replay slots)
  -> priority-tree leaf write + level recompute

Every op is a kernel on the caller's stream with static buffers, so the whole actor
step is captured into one hipGraph by :class:`apex_amd.engine.apex.ApexEngine`.
Actor ids are global (``actor_offset`` + local index) so the epsilon ladder spans
all shards of all ranks.
"""
from __future__ import annotations

import torch

from .. import ops
from ..algo.schedules import actor_epsilon
from .hbm_replay import HBMReplay

ENV_STATE_STRIDE = 32


class ActorShard:
    def __init__(self, replay: HBMReplay, n_envs: int, n_actions: int, n_step: int = 3, gamma: float = 0.99,
                 eps_base: float = 0.4, eps_alpha: float = 7.0, actor_offset: int = 0, total_actors: int | None = None,
                 seed: int = 0, mode: str = "reference", clip_rewards: bool = True, episode_life: bool = True,
                 max_episode_steps: int = 50000, action_repeat: int = 4, staged: int = 0):
        self.hip = ops.hip()
        self.replay = replay
        self.E, self.A, self.n = int(n_envs), int(n_actions), int(n_step)
        assert replay.n_envs == self.E, "replay slot layout is sized for this shard's env count"
        dev = replay.device
        self.device = dev
        self.seed = int(seed)
        E, A, n = self.E, self.A, self.n
        total = total_actors if total_actors is not None else E
        ids = torch.arange(actor_offset, actor_offset + E, dtype=torch.float64)
        self.eps = torch.as_tensor(actor_epsilon(ids.numpy(), total, eps_base, eps_alpha), dtype=torch.float32,
                                   device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.env_state = torch.zeros(E, ENV_STATE_STRIDE, **f32)
        self.new_frame = torch.zeros(E, **i32)
        self.ep_log = torch.zeros(E, 4, **f32)
        self.q = torch.zeros(E, A, **f32)
        self.actions = torch.zeros(E, **i32)
        self.reward = torch.zeros(E, **f32)
        self.done = torch.zeros(E, **f32)
        self.slot = torch.zeros(E, **i32)
        self.prio = torch.zeros(E, **f32)
        self.obs = torch.zeros(E, 4, 84, 84, dtype=torch.uint8, device=dev)
        self.step_counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.st = {
            "win_ids": torch.zeros(E, n, 4, **i32), "win_a": torch.zeros(E, n, **i32),
            "win_r": torch.zeros(E, n, **f32), "win_q": torch.zeros(E, n, A, **f32),
            "win_meta": torch.zeros(E, 4, **i32), "hist": torch.zeros(E, 4, **i32),
            "drain_ids": torch.zeros(E, n, 4, **i32), "drain_a": torch.zeros(E, n, **i32),
            "drain_r": torch.zeros(E, n, **f32), "drain_q": torch.zeros(E, n, **f32),
            "drain_meta": torch.zeros(E, 2, **i32), "drain_s2": torch.zeros(E, 4, **i32),
        }
        if mode not in ("reference", "textbook"):
            raise ValueError("mode must be 'reference' or 'textbook'")
        st_ptrs = {k: v.data_ptr() for k, v in self.st.items()}
        nmode = 0 if mode == "reference" else 1
        self.nstep = self.hip.make_nstep(E, A, n, replay.capacity, float(gamma), nmode, st_ptrs, replay.trans_ptrs())
        # staged mode (overlapped actor/learner streams): ``staged`` sets of [E] rows +
        # slots + priorities; the learner stream applies one half while the actor fills
        # the other
        self.staged = int(staged)
        if staged:
            self.stage = [{"s_ids": torch.zeros(E, 4, **i32), "s2_ids": torch.zeros(E, 4, **i32),
                           "action": torch.zeros(E, **i32), "reward": torch.zeros(E, **f32),
                           "done": torch.zeros(E, **f32)} for _ in range(self.staged)]
            self.stage_ptrs = [{k: v.data_ptr() for k, v in t.items()} for t in self.stage]
            self.stage_nstep = [self.hip.make_nstep(E, A, n, replay.capacity, float(gamma), nmode, st_ptrs, sp,
                                                    stage=1) for sp in self.stage_ptrs]
            self.stage_slot = [torch.zeros(E, **i32) for _ in range(self.staged)]
            self.stage_prio = [torch.zeros(E, **f32) for _ in range(self.staged)]
        self.env_params = self.hip.VecEnvParams(E, A, replay.frame_bytes, replay.frame_capacity, action_repeat,
                                                int(clip_rewards), int(episode_life), int(max_episode_steps))
        self.reset()

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def reset(self) -> None:
        self.hip.vec_env_reset(self.env_state.data_ptr(), self.seed, self.replay.frames.data_ptr(), self.env_params,
                               self.step_counter.data_ptr(), self.new_frame.data_ptr(), self.st["hist"].data_ptr(),
                               self.ep_log.data_ptr(), self._stream())

    def observe(self) -> torch.Tensor:
        """Current stacked observations u8 [E,4,84,84] (gathered from the frame ring)."""
        self.replay.gather_frames(self.st["hist"], self.obs)
        return self.obs

    def act_args(self) -> tuple:
        """(eps, rng seed, step counter, actions) pointers for an inference kernel that
        picks the actions itself (``heads_fwd_multi``'s eps-greedy epilogue: the same
        draw as ``select_actions``); then call :meth:`act_and_step` with ``selected=True``."""
        return (self.eps.data_ptr(), self.seed ^ 0x5E1EC7, self.step_counter.data_ptr(), self.actions.data_ptr())

    def act_and_step(self, q: torch.Tensor | None = None, parity: int | None = None, selected: bool = False,
                     tree: bool = True) -> None:
        """Given Q for the current observations (in ``self.q`` or ``q``), act, step the
        envs and push the emitted transitions into the replay (staged mode: into staging
        set ``parity``; :meth:`apply_staged` moves them into the replay).  ``selected``:
        ``self.actions`` already holds this step's eps-greedy actions (see :meth:`act_args`).
        ``tree=False``: rows only, no priority-tree write (a central actor rank's local mirror:
        the priorities travel in its packet to rank 0's tree)."""
        if q is not None and q.data_ptr() != self.q.data_ptr():
            self.q.copy_(q)
        s = self._stream()
        h = self.hip
        E, A = self.E, self.A
        if not selected:
            h.select_actions(self.q.data_ptr(), E, A, self.eps.data_ptr(), self.seed ^ 0x5E1EC7,
                             self.step_counter.data_ptr(), self.actions.data_ptr(), s)
        h.vec_env_step(self.env_state.data_ptr(), self.actions.data_ptr(), self.seed, self.step_counter.data_ptr(),
                       self.replay.frames.data_ptr(), self.env_params, self.reward.data_ptr(), self.done.data_ptr(),
                       self.new_frame.data_ptr(), self.ep_log.data_ptr(), s)
        if parity is not None:
            assert 0 <= parity < self.staged, "staging set out of range"
            h.nstep_emit(self.stage_nstep[parity], self.q.data_ptr(), self.actions.data_ptr(), self.reward.data_ptr(),
                         self.done.data_ptr(), self.new_frame.data_ptr(), self.step_counter.data_ptr(),
                         self.stage_slot[parity].data_ptr(), self.stage_prio[parity].data_ptr(), s, True)
            return  # the kernel advanced step_counter
        h.nstep_emit(self.nstep, self.q.data_ptr(), self.actions.data_ptr(), self.reward.data_ptr(),
                     self.done.data_ptr(), self.new_frame.data_ptr(), self.step_counter.data_ptr(),
                     self.slot.data_ptr(), self.prio.data_ptr(), s, not tree)  # (no tree: the kernel bumps)
        if tree:
            self.replay.write_batch(pre=(self.slot, self.prio, self.replay.filled), bump=self.step_counter)

    def apply_staged(self, parity: int) -> None:
        """Scatter staging set ``parity`` into the replay tables and write its
        priorities into the tree (the learner stream's half of a staged actor step)."""
        self.apply_rows(parity)
        self.apply_prios(parity)

    def apply_rows(self, parity: int) -> None:
        self.hip.apply_staged_rows(self.stage_ptrs[parity], self.replay.trans_ptrs(),
                                   self.stage_slot[parity].data_ptr(), self.stage_prio[parity].data_ptr(), self.E,
                                   self._stream())

    def apply_prios(self, parity: int) -> None:
        self.replay.write_batch(pre=self.staged_prio_write(parity))

    def staged_rows(self, parity: int) -> tuple:
        """``HBMReplay.sample_indices(rows=...)`` of staging set ``parity``."""
        return self.stage_ptrs[parity], self.stage_slot[parity], self.stage_prio[parity]

    def staged_prio_write(self, parity: int) -> tuple:
        """``HBMReplay.write_batch`` pre-write of staging set ``parity``: (slots, raw
        priorities, ``replay.filled`` advanced by E)."""
        return self.stage_slot[parity], self.stage_prio[parity], self.replay.filled

    def step(self, policy) -> None:
        """One full actor step with ``policy(obs_u8) -> Q f32 [E, A]``."""
        obs = self.observe()
        q = policy(obs)
        self.act_and_step(q)

    def episode_stats(self) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(last episode return, last episode length, finished episode count) per env."""
        return self.ep_log[:, 0], self.ep_log[:, 1], self.ep_log[:, 2]
