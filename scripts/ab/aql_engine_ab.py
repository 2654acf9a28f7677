#!/usr/bin/env python
"""Whole-engine A/B of AQLEngineConfig variants on one box: each variant is built, filled and
captured, then timed over ``--iters`` iterations, round-robin ``--rounds`` times (SGD steps/s,
the bench.py --algo aql metric).  ``python scripts/ab/aql_engine_ab.py fused_acting=0 fused_acting=1``"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+", help="comma-separated key=value overrides per variant ('-' = defaults)")
    ap.add_argument("--iters", type=int, default=250)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--env", default="BipedalWalker-v3")
    a = ap.parse_args()
    import torch

    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    engs = []
    for v in a.variants:
        kw = {}
        for item in ([] if v == "-" else v.split(",")):
            k, x = item.split("=")
            kw[k] = type(getattr(AQLEngineConfig, k))(int(x)) if isinstance(getattr(AQLEngineConfig, k), (bool, int)) \
                else type(getattr(AQLEngineConfig, k))(x)
        eng = AQLEngine(AQLEngineConfig(env_id=a.env, capacity=1_000_000, **kw), "cuda:0")
        eng.fill()
        eng.capture()
        for _ in range(20):
            eng.iteration()
        engs.append((v, eng))
    torch.cuda.synchronize()
    res = {v: [] for v, _ in engs}
    for _ in range(a.rounds):
        for v, eng in engs:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                eng.iteration()
            torch.cuda.synchronize()
            res[v].append(a.iters * eng.K / (time.perf_counter() - t0))
    for v, xs in res.items():
        print(f"{v:32s} " + " ".join(f"{x:8.0f}" for x in xs) + "  SGD steps/s")


if __name__ == "__main__":
    main()
