#!/usr/bin/env python
"""Wave-state table from scripts/gpu_pmc_waits.sh's two passes: where each kernel's wave
cycles go (SQ_WAIT_ANY parked on a waitcnt/barrier, SQ_WAIT_INST_ANY issue-stalled, the
active shares) and how much VALU runs beside the MFMAs.  SQ_* wave counters count
quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles (MI355X_MICROARCH.md)."""
import collections
import csv
import sys


def load(paths):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (file, dispatch) -> counter
    name = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            key = (p, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            name[key] = r["Kernel_Name"]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for key, cs in per.items():
        for c, v in cs.items():
            agg[name[key]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    m = load(sys.argv[1:])
    print("| kernel | wait (waitcnt/barrier) | issue-stalled | active | VALU active | LDS active | "
          "VALU / MFMA | MFMA-VALU coexec / MFMA busy |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for k, c in sorted(m.items()):
        if "SQ_WAVE_CYCLES" not in c or "SQ_INSTS_MFMA" not in c or not c.get("SQ_INSTS_MFMA"):
            continue
        wc = c["SQ_WAVE_CYCLES"]
        short = k.replace("(anonymous namespace)::", "").replace("apex::", "").split("(")[0][:64]
        print(f"| `{short}` | {c['SQ_WAIT_ANY'] / wc:.0%} | {c['SQ_WAIT_INST_ANY'] / wc:.0%} | "
              f"{c['SQ_ACTIVE_INST_ANY'] / wc:.0%} | {c['SQ_ACTIVE_INST_VALU'] / wc:.0%} | "
              f"{c['SQ_ACTIVE_INST_LDS'] / wc:.0%} | {c['SQ_INSTS_VALU'] / c['SQ_INSTS_MFMA']:.1f} | "
              f"{c['SQ_VALU_MFMA_COEXEC_CYCLES'] / max(1.0, c['SQ_VALU_MFMA_BUSY_CYCLES']):.0%} |")


if __name__ == "__main__":
    main()
