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
    ap.add_argument("--fused-step", type=int, default=1, help="one-launch step tail (aql_step_tail_k) or four")
    ap.add_argument("--bwd-tree", type=int, default=None, help="priority write in the backward launch (1) or not (0)")
    ap.add_argument("--fused-update", type=int, default=None, help="update launch after the gradients (1) or not")
    ap.add_argument("--levels-in-grad", type=int, default=None, help="tree levels in the gradient launch (1) or not")
    ap.add_argument("--halves", type=int, default=0, help="forward workgroup halves (0 default, 1, 2)")
    ap.add_argument("--groups", type=int, default=0, help="forward tile groups per sample (0: the launcher picks)")
    a = ap.parse_args()
    import torch

    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    cfg = AQLEngineConfig(env_id=a.env, capacity=1_000_000, fused_step=bool(a.fused_step))
    cfg.fwd_tile_groups = a.groups
    cfg.fwd_halves = a.halves
    if a.levels_in_grad is not None:
        cfg.tree_levels_in_grad = bool(a.levels_in_grad)
    if a.fused_update is not None:
        cfg.fused_update = bool(a.fused_update)
    if a.bwd_tree is not None:
        cfg.bwd_tree = bool(a.bwd_tree)
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
    print(f"fused_step={a.fused_step} {a.iters} learner steps: {1e6 * dt / a.iters:.1f} us/step", L.stats())
    if L.dbg is not None:  # APEX_AQL_DBG=1: backward phase timestamps (s_memtime cycles) of the last step
        d = L.dbg.cpu().tolist()
        print("bwd phase cycles:", [d[k + 1] - d[k] for k in range(7)], "total", d[7] - d[0])
        print("fwd phase cycles (staging, sampling, state load, encodings, adv1, out):",
              [d[k + 1] - d[k] for k in range(8, 14)], "total", d[14] - d[8])
        if d[16]:
            print("tree workgroup cycles (td, leaves, levels):", [d[k + 1] - d[k] for k in range(16, 19)],
                  "start after bwd start", d[16] - d[0])
            if d[24]:
                print("level walk cycles (dedup | level 1..):", d[24] - d[18],
                      [d[25 + k] - d[24 + k] for k in range(5) if d[25 + k]])


if __name__ == "__main__":
    main()
