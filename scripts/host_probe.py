"""Host-side cost of graph launches: time N replays of the captured learner / actor graphs
without synchronising (enqueue cost), then the GPU time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_amd.engine.apex import ApexEngine, EngineConfig  # noqa: E402
from apex_amd.engine.learner import LearnerConfig  # noqa: E402

cfg = EngineConfig(n_envs=256, replay_capacity=200_000, threshold_size=20_000, overlap=True,
                   learner=LearnerConfig(batch_size=512, forward="hip"))
eng = ApexEngine(cfg, "cuda")
eng.fill()
eng.capture()
for _ in range(20):
    eng.train_step()
torch.cuda.synchronize()
for name, fn in (("learner graph", lambda: eng._g_learn_a[0].replay()), ("actor graph", lambda: eng._g_actor[0].replay()),
                 ("train_step", eng.train_step)):
    N = 200
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tt = time.perf_counter() - t0
    print(f"{name:14s} host {1e6 * th / N:8.1f} us/launch   total {1e6 * tt / N:8.1f} us/launch", flush=True)
