"""Evaluator role (origin_repo/eval.py:19-108).

``N_ACTORS=N REPLAY_IP=... python -m apex_amd.roles.evaluator [flags]`` (rank 2 of
the role layout; ``N_EVAL=0`` runs without one).  Greedy (epsilon 0) on the
**unclipped**-reward env; after every episode it blocks for parameters newer than the
ones it played with, and logs ``evaluator/episode_reward`` /
``evaluator/episode_length``.  Exits when the learner sets the stop key.
"""
from __future__ import annotations

import argparse
import sys
import time

import numpy as np
import torch

from ..config import argparser
from ..models.dqn import DuelingDQN
from ..utils import set_global_seeds
from ..utils.tb import NullWriter, SummaryWriter
from .common import Heartbeat, ParamChannel, RoleLayout, init_role, load_model_flat_, make_role_env, stop_requested


class Evaluator:
    def __init__(self, cfg, writer=None, seed_offset=-1):
        seed = cfg.seed + seed_offset
        set_global_seeds(seed, use_torch=True)
        self.cfg = cfg
        self.env = make_role_env(cfg, clip_rewards=False, seed=seed)
        self.model = DuelingDQN(self.env)
        self.params = ParamChannel()
        self.version = 0
        self.writer = writer or NullWriter()
        self.returns: list[float] = []

    def _wait_params(self, timeout=600.0) -> bool:
        t0 = time.time()
        while True:
            try:
                v, flat = self.params.fetch(self.version)
            except (RuntimeError, OSError):  # store gone: the job is over
                return False
            if flat is not None:
                load_model_flat_(self.model, flat)
                self.version = v
                return True
            if stop_requested() or time.time() - t0 > timeout:
                return False
            time.sleep(0.05)

    def run(self, max_episodes: int = 0):
        if not self._wait_params():
            return self.returns
        ep_r, ep_len, ep_idx = 0.0, 0, 0
        state = self.env.reset()
        while True:
            action, _ = self.model.act(torch.as_tensor(np.asarray(state), dtype=torch.float32), 0.0)
            state, reward, done, _ = self.env.step(action)
            if ep_len % 1000 == 999 and stop_requested():
                break
            ep_r += reward
            ep_len += 1
            if done or ep_len == self.cfg.env.max_episode_length:
                state = self.env.reset()
                self.writer.add_scalar("evaluator/episode_reward", ep_r, ep_idx)
                self.writer.add_scalar("evaluator/episode_length", ep_len, ep_idx)
                self.returns.append(ep_r)
                ep_r, ep_len = 0.0, 0
                ep_idx += 1
                if (max_episodes and ep_idx >= max_episodes) or stop_requested():
                    break
                if not self._wait_params():
                    break
        return self.returns


def main(argv=None):
    extra = argparse.ArgumentParser(add_help=False)
    extra.add_argument("--max-episodes", type=int, default=0)
    extra.add_argument("--no-tb", action="store_true")
    ex, rest = extra.parse_known_args(sys.argv[1:] if argv is None else argv)
    args = argparser(rest)
    cfg = args.config
    layout = RoleLayout.from_env()
    rank = init_role("eval", layout, replay_ip=cfg.dist.replay_ip)
    hb = Heartbeat(rank)
    writer = NullWriter() if ex.no_tb else SummaryWriter(comment=f"-{cfg.env.env}-eval")
    out = Evaluator(cfg, writer).run(ex.max_episodes)
    writer.close()
    hb.stop()
    print(f"evaluator done: {len(out)} episodes", flush=True)
    return out


if __name__ == "__main__":
    main()
