#!/usr/bin/env python
"""Steady-state timeline stats of a rocprofv3 kernel trace: per learner step (marker to
marker), the union of kernel intervals (GPU busy with anything), per-queue busy time, and
idle gaps of the learner chain (kernels not in --actor-kernels)."""
import argparse
import csv


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="dqn_heads_bwd")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--actor-kernels", default="vec_env_step,select_actions,nstep_emit,copyBuffer,elementwise")
    ap.add_argument("--dump-step", action="store_true", help="print the kernels of the last full step")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"]]
    n = min(a.steps, len(marks) - 1)
    w0, w1 = marks[-n - 1], marks[-1]
    win = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows
           if w0 <= int(r["Start_Timestamp"]) < w1]
    step = (w1 - w0) / n / 1e3
    allu = union([(s, e) for s, e, _ in win]) / n / 1e3
    print(f"{n} steps: wall {step:.1f} us/step, GPU busy (union) {allu:.1f} us/step ({100 * allu / step:.0f}%)")
    qs = sorted({r.get("Queue_Id", "?") for _, _, r in win})
    for q in qs:
        u = union([(s, e) for s, e, r in win if r.get("Queue_Id", "?") == q]) / n / 1e3
        print(f"  queue {q}: busy {u:.1f} us/step")
    ak = a.actor_kernels.split(",")
    learner = [(s, e) for s, e, r in win if not any(k in r["Kernel_Name"] for k in ak)]
    print(f"  non-actor-named kernels busy (union) {union(learner) / n / 1e3:.1f} us/step")
    if a.dump_step:
        # Gantt of the last full step: offset/duration (us) per kernel, per queue, and the idle
        # gap before it on its queue (where that queue waits on another queue or the host).
        s0, s1 = marks[-2], marks[-1]
        ks = [(int(r["Start_Timestamp"]) - s0, int(r["End_Timestamp"]) - s0, r) for r in rows
              if s0 <= int(r["Start_Timestamp"]) < s1]
        last_end = {}
        print(f"\nstep gantt ({(s1 - s0) / 1e3:.1f} us): start  dur  gap-on-queue  queue  kernel")
        for s, e, r in ks:
            q = r.get("Queue_Id", "?")
            gap = s - last_end.get(q, s)
            last_end[q] = max(e, last_end.get(q, e))
            print(f"{s / 1e3:8.1f} {(e - s) / 1e3:6.1f} {gap / 1e3:7.1f}  q{q:>3}  {r['Kernel_Name'][:80]}")


if __name__ == "__main__":
    main()
