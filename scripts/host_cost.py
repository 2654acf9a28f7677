#!/usr/bin/env python
"""Host cost of one overlapped Ape-X train step, by part: actor / learner graph replays and
the event calls around them (bench.py's default engine, 1 GPU).  Prints microseconds per
call (median over --steps)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_amd.engine.apex import ApexEngine, EngineConfig, reserve_actor_stream  # noqa: E402
from apex_amd.engine.learner import LearnerConfig  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda", 0)
reserve_actor_stream(dev)
cfg = EngineConfig(n_envs=256, replay_capacity=2_000_000, threshold_size=50_000, overlap=True,
                   learner=LearnerConfig(batch_size=512, forward="hip", dtype="fp32"))
eng = ApexEngine(cfg, dev)
eng.fill()
eng.capture()
for _ in range(50):
    eng.train_step()
torch.cuda.synchronize(dev)
t = {"train_step": [], "actor_replay": [], "learner_replay": [], "events": []}
L = torch.cuda.current_stream(dev)
A = eng._astream
for i in range(steps):
    h = eng._half
    t0 = time.perf_counter()
    eng._ev_learn.block(A)
    t1 = time.perf_counter()
    with torch.cuda.stream(A):
        eng._g_actor[h].replay()
    t2 = time.perf_counter()
    eng._ev_actor[h].record(A)
    eng._ev_actor[1 - h].block(L)
    t3 = time.perf_counter()
    eng._g_learn_a[h].replay()
    t4 = time.perf_counter()
    eng._ev_learn.record(L)
    eng._half ^= 1
    t5 = time.perf_counter()
    t["events"].append((t1 - t0) + (t3 - t2) + (t5 - t4))
    t["actor_replay"].append(t2 - t1)
    t["learner_replay"].append(t4 - t3)
    if i % 50 == 0:
        torch.cuda.synchronize(dev)  # keep the queue short: measure the calls, not back-pressure
torch.cuda.synchronize(dev)
for _ in range(steps):
    t0 = time.perf_counter()
    eng.train_step()
    t["train_step"].append(time.perf_counter() - t0)
    if _ % 50 == 0:
        torch.cuda.synchronize(dev)
torch.cuda.synchronize(dev)
print({k: round(1e6 * statistics.median(v), 1) for k, v in t.items()}, flush=True)
print("graph nodes:", {"actor": eng._g_actor[0].raw_cuda_graph().num_nodes() if hasattr(eng._g_actor[0], "raw_cuda_graph") else None})
