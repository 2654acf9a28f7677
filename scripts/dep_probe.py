#!/usr/bin/env python
"""Upper bound of two-deep actor staging: bench.py's default engine timed with and
without the learner's wait on the previous actor step (the no-wait arm is NOT a valid
engine -- it races -- it only prices the dependency).  Prints steps/s for both arms."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_amd.engine.apex import ApexEngine, EngineConfig, reserve_actor_stream  # noqa: E402
from apex_amd.engine.learner import LearnerConfig  # noqa: E402


class NoWait:
    def __init__(self, ev):
        self.ev = ev

    def record(self, s):
        self.ev.record(s)

    def block(self, s):
        pass


def run(nowait: bool, steps: int = 2000) -> float:
    dev = torch.device("cuda", 0)
    cfg = EngineConfig(n_envs=256, replay_capacity=2_000_000, threshold_size=50_000, overlap=True,
                       learner=LearnerConfig(batch_size=512, forward="hip", dtype="fp32"))
    eng = ApexEngine(cfg, dev)
    eng.fill()
    eng.capture()
    if nowait:
        eng._ev_actor = [NoWait(e) for e in eng._ev_actor]
    for _ in range(50):
        eng.train_step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.train_step()
    torch.cuda.synchronize(dev)
    return steps / (time.perf_counter() - t0)


reserve_actor_stream(torch.device("cuda", 0))
print({"with_wait": round(run(False), 1), "no_wait": round(run(True), 1)}, flush=True)
