#!/usr/bin/env python
"""Phase stamps (s_memtime, shader cycles) of the AQL learner's backward launch: the
per-sample workgroup 0 (stamps 0-7) against the priority-tree workgroup (16-19, walk 24-29),
each read within its own workgroup (clocks of different CUs are not compared).  Eager steps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from apex_amd import ops  # noqa: E402


def main():
    h = ops.hip()
    dbg = torch.zeros(64, dtype=torch.int64, device="cuda:0")
    orig = h.make_aql_learn
    h.make_aql_learn = lambda on, tg, p, *a: orig(on, tg, dict(p, dbg=dbg.data_ptr()), *a)
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig

    eng = AQLEngine(AQLEngineConfig(env_id="BipedalWalker-v3", capacity=1_000_000), "cuda:0")
    eng.fill()
    L = eng.learner
    rows = []
    for k in range(12):
        dbg.zero_()
        L.step(drawn=k > 0, draw_next=True)
        torch.cuda.synchronize()
        rows.append(dbg.cpu().tolist())
    for r in rows[-4:]:
        samp = [r[i + 1] - r[i] for i in range(7) if r[i] and r[i + 1]]
        tree = [r[17 + i] - r[16 + i] for i in range(3) if r[16 + i] and r[17 + i]]
        walk = [r[25 + i] - r[24 + i] for i in range(5) if r[24 + i] and r[25 + i]]
        print("sample wg phases", samp, "total", sum(samp), "| tree wg", tree, "total", sum(tree), "| walk", walk,
              "| fwd stamps", [r[i + 1] - r[i] for i in range(8, 14) if r[i] and r[i + 1]])


if __name__ == "__main__":
    main()
