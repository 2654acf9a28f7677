"""Actor-side n-step batcher with actor-computed initial priorities
(reference memory.py:393-478).

``BatchStorage(n_steps, gamma, mode="reference")`` reproduces the reference exactly:

* Q1  emission happens when the window already holds n states, and the *current*
  reward is folded in: R = r_{t-n} + ... + gamma^n r_t (n+1 rewards) with the
  bootstrap state s_t;
* Q2  on ``done`` only the oldest window entry is emitted, with next-state = the
  pre-terminal state passed to ``add``; the remaining tail is dropped;
* Q3  the Q-value window is not cleared on ``done`` (stale Q for short episodes);
* Q4  an episode whose first step is terminal raised IndexError in the reference;
  here it emits nothing.

``mode="textbook"`` is the corrected n-step: R = sum_{i<n} gamma^i r_{t-n+i},
next-state s_t, bootstrap gamma^n max_a Q(s_t); on ``done`` every remaining window
entry is flushed as terminal and all windows (Q included) are cleared.

Priority = |R + gamma^n * max_a Q_next * (1 - d) - Q(s_0, a_0)| + 1e-6 computed from
the actor's own Q values (no target net, no double-Q).  The GPU equivalent for
vectorised actors is the ``nstep_emit`` kernel (``apex_amd.engine``).
"""
from __future__ import annotations

from collections import deque

import numpy as np


class BatchStorage:
    MODES = ("reference", "textbook")

    def __init__(self, n_steps, gamma=0.99, mode: str = "reference"):
        if mode not in self.MODES:
            raise ValueError(f"mode must be one of {self.MODES}")
        self.n_steps = int(n_steps)
        self.gamma = gamma
        self.mode = mode
        self.state_deque = deque(maxlen=self.n_steps)
        self.action_deque = deque(maxlen=self.n_steps)
        self.reward_deque = deque(maxlen=self.n_steps)
        self.q_values_deque = deque(maxlen=self.n_steps)
        self.reset()

    def reset(self):
        self.states, self.actions, self.rewards = [], [], []
        self.next_states, self.dones = [], []
        self.q_values, self.next_q_values = [], []

    def _emit(self, s0, a0, ret, q0, s_next, q_next, done):
        self.states.append(s0)
        self.actions.append(a0)
        self.rewards.append(ret)
        self.next_states.append(s_next)
        self.dones.append(np.float32(done))
        self.q_values.append(q0)
        self.next_q_values.append(q_next)

    def add(self, state, reward, action, done, q_values):
        if self.mode == "reference":
            self._add_reference(state, reward, action, done, q_values)
        else:
            self._add_textbook(state, reward, action, done, q_values)

    def _add_reference(self, state, reward, action, done, q_values):
        if (len(self.state_deque) == self.n_steps or done) and len(self.state_deque) > 0:
            ret = self.multi_step_reward(*self.reward_deque, reward)
            self._emit(self.state_deque[0], self.action_deque[0], ret, self.q_values_deque[0], state, q_values, done)
        if done:
            self.state_deque.clear()
            self.reward_deque.clear()
            self.action_deque.clear()
        else:
            self.state_deque.append(state)
            self.reward_deque.append(reward)
            self.action_deque.append(action)
            self.q_values_deque.append(q_values)

    def _add_textbook(self, state, reward, action, done, q_values):
        if len(self.state_deque) == self.n_steps:
            ret = self.multi_step_reward(*self.reward_deque)
            self._emit(self.state_deque[0], self.action_deque[0], ret, self.q_values_deque[0], state, q_values, False)
            self.state_deque.popleft()
            self.reward_deque.popleft()
            self.action_deque.popleft()
            self.q_values_deque.popleft()
        self.state_deque.append(state)
        self.reward_deque.append(reward)
        self.action_deque.append(action)
        self.q_values_deque.append(q_values)
        if done:
            zeros = np.zeros_like(np.asarray(q_values, dtype=np.float32))
            rs = list(self.reward_deque)
            for j in range(len(self.state_deque)):
                ret = self.multi_step_reward(*rs[j:])
                self._emit(self.state_deque[j], self.action_deque[j], ret, self.q_values_deque[j], state, zeros, True)
            self.state_deque.clear()
            self.reward_deque.clear()
            self.action_deque.clear()
            self.q_values_deque.clear()

    def compute_priorities(self):
        if not self.states:
            return np.zeros(0, dtype=np.float64)
        actions = np.asarray(self.actions)
        rewards = np.asarray(self.rewards, dtype=np.float64)
        dones = np.asarray(self.dones, dtype=np.float64)
        q = np.stack(self.q_values)
        q_next = np.stack(self.next_q_values)
        q_a = q[np.arange(len(q)), actions]
        target = rewards + (self.gamma ** self.n_steps) * q_next.max(1) * (1 - dones)
        return np.abs(target - q_a) + 1e-6

    def make_batch(self):
        prios = self.compute_priorities()
        return [self.states, self.actions, self.rewards, self.next_states, self.dones], prios

    def multi_step_reward(self, *rewards):
        ret = 0.0
        for i, r in enumerate(rewards):
            ret += r * (self.gamma ** i)
        return ret

    def __len__(self):
        return len(self.states)
