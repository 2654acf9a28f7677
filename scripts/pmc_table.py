#!/usr/bin/env python
"""Per-kernel mean of rocprofv3 --pmc counter_collection CSVs (one or more passes)."""
import collections
import csv
import sys


def derived(acc, name_of):
    """Per-kernel summary: wall us (GRBM_GUI_ACTIVE / 8 XCDs at 2.4 GHz), MFMA busy share of
    every SIMD's cycles (256 CUs x 4 SIMDs), VALU and LDS instructions per MFMA, LDS bank
    conflict cycles per active LDS cycle, L2 hit rate, HBM fetch MB."""
    def m(d, c):
        per = collections.defaultdict(float)
        for (disp, _), v in d.get(c, []):
            per[disp] += v
        return sum(per.values()) / max(1, len(per)) if per else float("nan")
    print("| kernel | us | MFMA busy | VALU / MFMA | LDS insts / MFMA | LDS conflict / LDS active | L2 hit | fetch MB |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for k, d in acc.items():
        cyc = m(d, "GRBM_GUI_ACTIVE") / 8.0
        mf = m(d, "SQ_INSTS_MFMA")
        if not mf or mf != mf:
            continue
        busy = m(d, "SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024.0)
        hit, miss = m(d, "TCC_HIT_sum"), m(d, "TCC_MISS_sum")
        print(f"| `{k}` | {cyc / 2400.0:.1f} | {100 * busy:.0f}% | {m(d, 'SQ_INSTS_VALU') / mf:.2f} | "
              f"{m(d, 'SQ_INSTS_LDS') / mf:.2f} | {m(d, 'SQ_LDS_BANK_CONFLICT') / max(1.0, m(d, 'SQ_ACTIVE_INST_LDS')):.2f} | "
              f"{100 * hit / max(1.0, hit + miss):.0f}% | {m(d, 'FETCH_SIZE') / 1024.0:.1f} |")


def main(paths, summary=False):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("apex::", "")
            k = (k[5:] if k.startswith("void ") else k).split("(")[0][:70]
            key = (r.get("Dispatch_Id"), r["Counter_Name"])
            acc[k][r["Counter_Name"]].append((key, float(r["Counter_Value"])))
    if summary:
        return derived(acc, None)
    names = sorted({c for k in acc for c in acc[k]})
    print("| kernel | " + " | ".join(names) + " |")
    print("|---|" + "---:|" * len(names))
    for k, d in acc.items():
        row = []
        for c in names:
            # sum over dimensions (XCD/SE instances) per dispatch, then mean over dispatches
            per = collections.defaultdict(float)
            for (disp, _), v in d.get(c, []):
                per[disp] += v
            row.append(f"{sum(per.values()) / max(1, len(per)):.4g}" if per else "")
        print(f"| `{k}` | " + " | ".join(row) + " |")


if __name__ == "__main__":
    args = sys.argv[1:]
    main([a for a in args if a != "--summary"], summary="--summary" in args)
