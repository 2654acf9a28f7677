#!/usr/bin/env python
"""Per-kernel steady-state table from a rocprofv3 rocpd database (``-d DIR`` run with
``--kernel-trace``): groups dispatches by (kernel, grid size) over the last ``--steps``
learner steps (a step = one ``--marker`` kernel dispatch) and prints a markdown table of
calls/step, mean duration and the share of the summed kernel time.  ``--flops`` adds
achieved TFLOP/s for kernels named in a JSON {substring: flop per call} map."""
import argparse
import collections
import json
import sqlite3


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("apex::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="dqn_heads_bwd_k")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--flops", default=None, help="JSON map {name substring: flop per call}")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x, queue_id from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 2:
        raise SystemExit(f"marker {a.marker!r} found {len(marks)} times")
    lo = marks[max(0, len(marks) - 1 - a.steps)]
    hi = marks[-1]
    nsteps = len([m for m in marks if lo <= m < hi])
    sel = rows[lo:hi]
    t_wall = (rows[hi][1] - rows[lo][1]) / nsteps / 1e3
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e, gx, wx, q in sel:
        k = (short(name), gx // max(wx, 1))
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    total = sum(v[1] for v in agg.values())
    flops = json.loads(a.flops) if a.flops else {}
    print(f"steady state: {nsteps} steps, wall {t_wall:.1f} us/step (marker to marker), "
          f"summed kernel time {total / nsteps:.1f} us/step\n")
    print("| kernel | workgroups | calls/step | mean us | us/step | share | TFLOP/s |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for (name, wg), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        tf = ""
        for sub, f in flops.items():
            if sub in name and n:
                tf = f"{f / (t / n * 1e-6) / 1e12:.1f}"
        print(f"| {name} | {wg} | {n / nsteps:.2f} | {t / n:.2f} | {t / nsteps:.2f} | {100 * t / total:.1f}% | {tf} |")


if __name__ == "__main__":
    main()
