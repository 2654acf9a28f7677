#!/usr/bin/env python
"""Whole-step A/B of single-GPU Ape-X bench variants on ONE box, alternated: each variant is a
fresh ``bench.py`` process (the bench config: fp32 DQN, batch 512, 256 envs, overlapped actor),
run round-robin ``--rounds`` times; prints learner steps/s per variant (median and every round)
as one JSON line.

A variant is a comma-separated list of overrides ('-' = the defaults):
  ss=MASK        APEX_F32_STAGE_SPLIT: f32 GEMM forms, forward + 4 x backward pairs
                 (0 register split, 1 stage-split, 2 stage-split single LDS image, 3 = 2 at >= 3 waves/SIMD)
  env:NAME=VAL   any other environment variable
  arg:--flag[=VAL]  a bench.py flag (e.g. arg:--actor-at=loss)
e.g. ``python scripts/ab/apex_engine_ab.py - ss=4 ss=8 ss=8,arg:--actor-at=loss``.

Separate processes on purpose: several engines in one process draw their actor / tree streams
from torch's pool, which spreads them over the GPU's 4 hardware queues round-robin -- an
engine whose actor stream shares the learner's queue serialises (0.51 vs 0.31 ms per step,
engine/apex.py reserve_actor_stream), which made a one-process A/B read 20 % differences that
were queue placement, not kernels."""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(variant: str, steps: int, warmup: int, timeout: float) -> float:
    env = dict(os.environ)
    flags = []
    for item in ([] if variant == "-" else variant.split(",")):
        if item.startswith("ss="):
            env["APEX_F32_STAGE_SPLIT"] = item[3:]
        elif item.startswith("env:"):
            k, v = item[4:].split("=", 1)
            env[k] = v
        elif item.startswith("arg:"):
            flags += item[4:].split("=", 1)
        else:
            raise SystemExit(f"bad variant item {item!r}")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", str(warmup), *flags]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    if out.returncode != 0:
        raise SystemExit(f"{variant}: bench.py exited {out.returncode}\n{out.stderr[-2000:]}")
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    return float(json.loads(line)["value"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=240.0)
    a = ap.parse_args()
    res = {v: [] for v in a.variants}
    for rnd in range(a.rounds):
        for v in a.variants:
            res[v].append(run(v, a.steps, a.warmup, a.timeout))
            print(f"round {rnd} {v}: {res[v][-1]:.1f}", flush=True)
    print(json.dumps({"steps_per_s_median": {v: round(statistics.median(x), 1) for v, x in res.items()},
                      "rounds": {v: [round(y, 1) for y in x] for v, x in res.items()}, "steps": a.steps}))


if __name__ == "__main__":
    main()
