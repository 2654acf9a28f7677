#!/usr/bin/env python
"""Per-step GPU time of the first steps after ApexEngine.capture() (events around each
train_step, no host sync in between): how many replays until steady state."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=256, replay_capacity=2_000_000, threshold_size=50_000, overlap=True,
                       learner=LearnerConfig(batch_size=512, forward="hip", dtype="fp32"))
    eng = ApexEngine(cfg, "cuda:0")
    eng.fill(cfg.threshold_size)
    eng.capture()
    torch.cuda.synchronize()
    n = 80
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    ev[0].record()
    for i in range(n):
        eng.train_step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    print("per-step ms:", " ".join(f"{x:.3f}" for x in ms))
    for a, b in ((0, 5), (5, 25), (25, 50), (50, 80)):
        print(f"steps {a}-{b}: mean {sum(ms[a:b]) / (b - a):.4f} ms")
    import time
    for idle in (0.05, 1.0):  # after an idle gap: does the slow start come back (clock / power state)?
        time.sleep(idle)
        ev[0].record()
        for i in range(30):
            eng.train_step()
            ev[i + 1].record()
        torch.cuda.synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(30)]
        print(f"after {idle:.2f} s idle: steps 0-5 {sum(ms[:5]) / 5:.4f}  5-25 {sum(ms[5:25]) / 20:.4f}  "
              f"25-30 {sum(ms[25:30]) / 5:.4f} ms")


if __name__ == "__main__":
    main()
