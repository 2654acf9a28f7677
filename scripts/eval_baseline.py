#!/usr/bin/env python
"""Return of the uniform-random policy (epsilon 1) and of a random-init greedy network on
the synthetic game, measured with the GPU evaluator's settings (unclipped rewards,
episodic life, 18 actions): the reference points for the learning curve of train.py."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_amd.engine.evaluator import GPUEvaluator  # noqa: E402
from apex_amd.models.dqn import DuelingDQN  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", type=int, default=64)
ap.add_argument("--steps", type=int, default=3000)
a = ap.parse_args()
dev = torch.device("cuda")
torch.manual_seed(1122)
m = DuelingDQN.from_shapes((4, 84, 84), 18).to(dev)
out = {}
for name, eps in (("random_policy", 1.0), ("random_init_greedy", 0.0)):
    ev = GPUEvaluator(m, a.envs, 18, device=dev, seed=99, epsilon=eps)
    rets = []
    for i in range(a.steps):
        ev.step()
        if i % 100 == 99:
            rets += [r for r, _ in ev.poll()]
    rets += [r for r, _ in ev.poll()]
    out[name] = {"episodes": len(rets), "mean_return": sum(rets) / max(1, len(rets))}
print(json.dumps(out))
