"""Exploration / IS schedules used across the reference trainers.

* Ape-X epsilon ladder: eps_i = eps_base^(1 + i/(N-1) * eps_alpha)
  (origin_repo/actor.py:69, batchrecorder.py:121).  N = 1 divides by zero in the
  reference; here eps_0 = eps_base.
* PER beta annealing: beta(t) = min(1, beta0 + t (1 - beta0) / horizon)
  (ApeX.py:39 horizon 1000, DQN.py:40, AQL.py:51 horizon max_step).
* DQN epsilon decay: eps(t) = eps_final + (eps_start - eps_final) exp(-t / decay)
  (DQN.py:41).
"""
from __future__ import annotations

import math

import numpy as np


def actor_epsilon(actor_id, n_actors: int, eps_base: float = 0.4, eps_alpha: float = 7.0):
    if n_actors <= 1:
        return np.full(np.shape(actor_id), eps_base, dtype=np.float64) if np.ndim(actor_id) else float(eps_base)
    return eps_base ** (1 + np.asarray(actor_id, dtype=np.float64) / (n_actors - 1) * eps_alpha) \
        if np.ndim(actor_id) else eps_base ** (1 + actor_id / (n_actors - 1) * eps_alpha)


def beta_by_frame(frame_idx: int, beta_start: float = 0.4, horizon: float = 1000.0) -> float:
    return min(1.0, beta_start + frame_idx * (1.0 - beta_start) / horizon)


def epsilon_by_frame(frame_idx: int, eps_start: float = 1.0, eps_final: float = 0.01, decay: float = 500.0) -> float:
    return eps_final + (eps_start - eps_final) * math.exp(-1.0 * frame_idx / decay)


def step_scheduler_early(scheduler) -> None:
    """``scheduler.step()`` before ``optimizer.step()`` (the reference decays
    the LR one step early, ApeX.py:60-61 / DQN.py:71-73); torch's ordering warning is
    expected here and silenced."""
    import re
    import warnings

    with warnings.catch_warnings():
        # ``message`` is a regex: escape the parentheses of "step()"
        warnings.filterwarnings("ignore", message=re.escape("Detected call of `lr_scheduler.step()`"))
        scheduler.step()
