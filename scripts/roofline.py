#!/usr/bin/env python
"""Roofline table of the Ape-X DQN step from a rocprofv3 kernel-trace CSV.

Per kernel (name, workgroups): calls/step and mean duration over the last ``--steps``
learner steps (marker to marker), the FLOP of each launch from the Nature-CNN dueling
network's shapes (samples inferred from the grid), achieved TFLOP/s and % of the MI355X
peak of the step's precision (fp32 MFMA 157.3 TF, bf16 2.5 PF dense), and the time share.
Memory-bound kernels (optimizer, finalize, replay) get their modelled HBM bytes and GB/s
against 8 TB/s.  Usage: ``roofline.py TRACE.csv [--dtype fp32] [--batch 512] [--envs 256]``.
"""
import argparse
import collections
import csv

PEAK_TF = {"fp32": 157.3, "bf16": 2500.0}
HBM_GBS = 8000.0
# per-sample forward FLOP of each layer (2 * MACs)
CONV1 = 20 * 20 * 32 * (4 * 8 * 8) * 2
CONV2 = 9 * 9 * 64 * (32 * 4 * 4) * 2
CONV3 = 7 * 7 * 64 * (64 * 3 * 3) * 2
FC1 = 3136 * 256 * 2
N_PARAMS = 32 * 256 + 32 + 64 * 512 + 64 + 64 * 576 + 64 + 2 * (3136 * 128 + 128) + 128 * 18 + 18 + 128 + 1


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("apex::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def model(name, wgs, B, E):
    """(flop, bytes) of one launch, or (None, None) if unmodelled."""
    if "conv1_fwd_x3_k" in name:  # persistent: grid = min(samples, 512)
        return (3 * B if wgs >= 512 else E) * CONV1, None
    if "conv1_fwd_k" in name:
        return wgs * CONV1, None  # one workgroup per (problem, sample)
    if "Conv2Fwd" in name:
        return (3 * B if wgs > 1000 else E) * CONV2, None
    if "Conv3Fwd" in name:
        return (3 * B if wgs > 600 else E) * CONV3, None
    if "Fc1Fwd" in name or "fc1_fwd" in name:
        return (3 * B if wgs > 300 else E) * FC1, None  # learner 336 (128x64) | 672 (64x64) wg
    if "Fc1Wgrad" in name or "fc1_bwd" in name:
        return 2 * B * FC1, None  # weight + input gradient
    if "ConvWgrad<3>" in name:
        return 2 * B * CONV3, None
    if "ConvWgrad<2>" in name:
        return 2 * B * CONV2, None
    if "conv1_wgrad" in name:
        return B * CONV1, None
    if "opt_step_k" in name:
        return None, N_PARAMS * 4 * 8  # p, g, s1, s2 read + p, s1, s2 + packed copy written
    if "grad_finalize_k" in name:
        return None, None
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="dqn_heads_bwd")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--envs", type=int, default=256)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"]]
    n = min(a.steps, len(marks) - 1)
    w0, w1 = marks[-n - 1], marks[-1]
    agg = collections.defaultdict(list)
    for r in rows:
        s = int(r["Start_Timestamp"])
        if w0 <= s < w1:
            wg = (int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) // max(
                1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
            agg[(short(r["Kernel_Name"]), wg)].append((int(r["End_Timestamp"]) - s) / 1e3)
    step_us = (w1 - w0) / n / 1e3
    total = sum(sum(v) for v in agg.values()) / n
    peak = PEAK_TF[a.dtype]
    print(f"steady state: {n} steps, wall {step_us:.1f} us/step, summed kernel time {total:.1f} us/step, "
          f"peak {peak} TF ({a.dtype}), HBM {HBM_GBS / 1000:.0f} TB/s")
    print()
    print("| kernel | workgroups | calls/step | mean us | us/step | share | GFLOP/call | TFLOP/s | % peak | GB/s |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    flop_step = 0.0
    for (k, wg), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        mean = sum(v) / len(v)
        per = sum(v) / n
        if per < 0.2:
            continue
        f, b = model(k, wg, a.batch, a.envs)
        tf = pct = gbs = ""
        gf = ""
        if f:
            gf = f"{f / 1e9:.3f}"
            tf = f"{f / mean / 1e6:.1f}"
            pct = f"{100 * f / mean / 1e6 / peak:.0f}%"
            flop_step += f * len(v) / n
        if b:
            gbs = f"{b / mean / 1e3:.0f}"
        print(f"| {k[:60]} | {wg} | {len(v) / n:.2f} | {mean:.2f} | {per:.2f} | {100 * per / total:.1f}% | {gf} | "
              f"{tf} | {pct} | {gbs} |")
    print()
    print(f"modelled FLOP per step {flop_step / 1e9:.2f} GFLOP -> {flop_step / step_us / 1e6:.1f} TFLOP/s over the "
          f"wall step ({100 * flop_step / step_us / 1e6 / peak:.0f}% of {a.dtype} peak)")


if __name__ == "__main__":
    main()
