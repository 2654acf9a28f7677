#!/usr/bin/env python
"""AQL learner-step microbenchmark (rocprofv3 / PMC target): builds the GPU AQL engine,
fills the replay and runs ``--iters`` learner steps (optionally as one captured graph)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="BipedalWalker-v3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--fused", type=int, default=1, help="the four-launch step (1) or the reference sequence (0)")
    ap.add_argument("--groups", type=int, default=0, help="forward tile groups per sample (0: the launcher picks)")
    a = ap.parse_args()
    import torch

    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    cfg = AQLEngineConfig(env_id=a.env, capacity=1_000_000, fused=bool(a.fused), fwd_tile_groups=a.groups)
    eng = AQLEngine(cfg, "cuda:0")
    eng.fill(4096)
    L = eng.learner
    L.step()
    torch.cuda.synchronize()
    pre = L.predraw  # the engine's schedule: each step draws the next one's rows

    def steps():
        for k in range(a.iters):
            L.step(drawn=pre and k > 0, draw_next=pre and k + 1 < a.iters)

    if a.graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            steps()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
    else:
        t0 = time.perf_counter()
        steps()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"fused={a.fused} {a.iters} learner steps: {1e6 * dt / a.iters:.1f} us/step", L.stats())


if __name__ == "__main__":
    main()
