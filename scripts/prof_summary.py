#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace into per-learner-step kernel time.

Usage: python scripts/prof_summary.py gpurun_out/prof_x/run_kernel_trace.csv [--marker dqn_loss] [--steps 40]
Steady state = the last ``--steps`` intervals between consecutive ``--marker`` kernel
launches (one marker per learner step).  Prints a markdown table.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="dqn_loss")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [r for r in rows if a.marker in r["Kernel_Name"]]
    n = min(a.steps, len(marks) - 1)
    w0, w1 = int(marks[-n - 1]["Start_Timestamp"]), int(marks[-1]["Start_Timestamp"])
    win = [r for r in rows if w0 <= int(r["Start_Timestamp"]) < w1]
    dur = collections.defaultdict(float)
    cnt = collections.Counter()
    meta = {}
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = r["Kernel_Name"]
        dur[k] += d
        cnt[k] += 1
        meta[k] = (r.get("VGPR_Count"), r.get("LDS_Block_Size"), r.get("Grid_Size_X"), r.get("Workgroup_Size_X"))
    busy = sum(dur.values())
    print(f"steady state over {n} learner steps: wall {(w1 - w0) / n / 1e3:.1f} us/step, "
          f"kernel busy {busy / n / 1e3:.1f} us/step, {len(win) / n:.1f} kernels/step\n")
    print("| us/step | calls/step | share | VGPR | LDS B | grid | wg | kernel |")
    print("|---:|---:|---:|---:|---:|---:|---:|---|")
    for k, v in sorted(dur.items(), key=lambda x: -x[1])[:a.top]:
        vg, lds, gx, wg = meta[k]
        print(f"| {v / n / 1e3:.1f} | {cnt[k] / n:.1f} | {100 * v / busy:.1f}% | {vg} | {lds} | {gx} | {wg} | "
              f"`{k[:90]}` |")


if __name__ == "__main__":
    main()
