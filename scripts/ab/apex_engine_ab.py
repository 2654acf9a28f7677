#!/usr/bin/env python
"""Whole-step A/B of single-GPU Ape-X engine variants on ONE box, interleaved: every variant
is built, filled and captured in this process (the bench config: fp32 DQN, batch 512, 256
envs, overlapped actor), then timed over ``--steps`` train steps, round-robin ``--rounds``
times; prints learner steps/s per variant (median and every round) as one JSON line.

A variant is a comma-separated list of overrides ('-' = the defaults):
  actor_at=start|loss     EngineConfig.actor_at
  ss=MASK                 f32 GEMM forms at capture time, forward + 4 x backward pairs
                          (0 register split, 1 stage-split, 2 stage-split single LDS image;
                          f32_set_stage_split)
  <EngineConfig field>=int
e.g. ``python scripts/ab/apex_engine_ab.py ss=0 ss=8 ss=10 ss=8,actor_at=loss``.  Interleaving
removes the 2-5 % box-to-box and clock-ramp differences a sequence of bench runs carries."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--capacity", type=int, default=2_000_000)
    ap.add_argument("--threshold", type=int, default=50_000)
    a = ap.parse_args()
    import torch

    from apex_amd import ops
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    hip = ops.hip()
    dev = torch.device("cuda", 0)
    engs = []
    for v in a.variants:
        kw, ss = {}, hip.f32_stage_split()
        for item in ([] if v == "-" else v.split(",")):
            k, x = item.split("=")
            if k == "ss":
                ss = int(x)
            elif k == "actor_at":
                kw[k] = x
            else:
                kw[k] = int(x)
        hip.f32_set_stage_split(ss)
        cfg = EngineConfig(n_envs=256, replay_capacity=a.capacity, threshold_size=a.threshold, overlap=True,
                           learner=LearnerConfig(batch_size=512, forward="hip", dtype="fp32"), **kw)
        eng = ApexEngine(cfg, dev)
        eng.fill()
        eng.capture(warm_replays=100)
        torch.cuda.synchronize()
        engs.append((v, eng))
        print(f"built {v} (stage split {ss})", flush=True)
    res = {v: [] for v, _ in engs}
    for rnd in range(a.rounds):
        for v, eng in engs:
            for _ in range(100):  # re-warm after the other variants ran
                eng.train_step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                eng.train_step()
            torch.cuda.synchronize()
            res[v].append(a.steps / (time.perf_counter() - t0))
        print(f"round {rnd}: " + ", ".join(f"{v} {res[v][-1]:.1f}" for v, _ in engs), flush=True)
    print(json.dumps({"steps_per_s_median": {v: round(statistics.median(x), 1) for v, x in res.items()},
                      "rounds": {v: [round(y, 1) for y in x] for v, x in res.items()}, "steps": a.steps}))


if __name__ == "__main__":
    main()
