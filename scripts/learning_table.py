#!/usr/bin/env python
"""train.py log -> the learning-curve markdown table (one row per ``Step:`` log line).

``python scripts/learning_table.py gpurun_out/learn/train.log [baseline.json]``

Columns: learner step, loss, greedy return of the evaluator episodes that finished in the row's
window (eps 0, unclipped rewards: origin_repo/eval.py), how many of them ended at the step cap,
the mean return so far of the evaluator episodes still running at the log line (the explicit
marker when none finished), the actor's clipped episodic-life return, learner steps/s."""
import json
import re
import sys


def parse(path):
    rows = []
    for line in open(path, errors="replace"):
        m = re.match(r"Step: (\d+) (.*)", line.strip())
        if not m:
            continue
        kv = dict(re.findall(r"(\S+)=(\S+)", m.group(2)))
        rows.append((int(m.group(1)), {k: float(v) for k, v in kv.items()}))
    return rows


def fmt(x, nd=4):
    return "-" if x is None else f"{x:.{nd}g}"


def main():
    rows = parse(sys.argv[1])
    if len(sys.argv) > 2:
        b = json.load(open(sys.argv[2]))
        print(f"Baselines (scripts/eval_baseline.py): {b}\n")
    print("| learner step | loss | greedy return (finished) | capped | greedy running return (in progress) "
          "| actor return | learner steps/s |")
    print("|---:|---:|---:|---:|---:|---:|---:|")
    for step, d in rows:
        print(f"| {step} | {fmt(d.get('learner/loss'))} | {fmt(d.get('evaluator/episode_reward'))} | "
              f"{fmt(d.get('evaluator/capped_episodes'), 3)} | {fmt(d.get('evaluator/running_return'))} | "
              f"{fmt(d.get('actor/episode_reward'))} | {fmt(d.get('learner/BPS'))} |")


if __name__ == "__main__":
    main()
