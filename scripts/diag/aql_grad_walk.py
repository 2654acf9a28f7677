#!/usr/bin/env python
"""Time the AQL gradient launch with and without its tree-walk workgroup (levels 2..): the
contraction alone (the step's plain AqlGrad handle) vs the handle with the walk, each replayed
in a captured graph of 200 launches after one real learner step (timing only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    eng = AQLEngine(AQLEngineConfig(env_id="BipedalWalker-v3", capacity=1_000_000), "cuda:0")
    eng.fill()
    L = eng.learner
    L.step()
    torch.cuda.synchronize()
    h, s = L.hip, torch.cuda.current_stream().cuda_stream
    res = {}
    for name, G in (("contraction only", L.G), ("contraction + walk (levels 2..)", L.G_levels)):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(200):
                h.aql_grad(G, torch.cuda.current_stream().cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = 1000 * e0.elapsed_time(e1) / 200
    for k, v in res.items():
        print(f"{k}: {v:.2f} us per launch")


if __name__ == "__main__":
    main()
