"""Play a saved checkpoint greedily (origin_repo/enjoy.py:18-48).

``python -m apex_amd.roles.enjoy [--render] [--model model.pth] [--episodes N] [flags]``

Loads the reference-format ``state_dict`` with ``torch.load(weights_only=True)`` on
the CPU and prints "Episode Length / Reward" per episode on the unclipped env.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np
import torch

from ..config import argparser
from ..models.dqn import DuelingDQN
from ..utils import set_global_seeds
from ..utils.checkpoint import load_model
from .common import make_role_env


def play(cfg, model_path="model.pth", episodes=0, render=False):
    seed = cfg.seed + 1122
    set_global_seeds(seed, use_torch=True)
    env = make_role_env(cfg, clip_rewards=False, seed=seed)
    model = load_model(DuelingDQN(env), model_path)
    results = []
    ep_r, ep_len = 0.0, 0
    state = env.reset()
    while True:
        if render:
            env.render()
        action, _ = model.act(torch.as_tensor(np.asarray(state), dtype=torch.float32), 0.0)
        state, reward, done, _ = env.step(action)
        ep_r += reward
        ep_len += 1
        if done:
            state = env.reset()
            print(f"Episode Length / Reward: {ep_len} / {ep_r}", flush=True)
            results.append((ep_len, ep_r))
            ep_r, ep_len = 0.0, 0
            if episodes and len(results) >= episodes:
                return results


def main(argv=None):
    extra = argparse.ArgumentParser(add_help=False)
    extra.add_argument("--model", default="model.pth")
    extra.add_argument("--episodes", type=int, default=0)
    ex, rest = extra.parse_known_args(sys.argv[1:] if argv is None else argv)
    args = argparser(rest)
    return play(args.config, ex.model, ex.episodes, args.render)


if __name__ == "__main__":
    main()
