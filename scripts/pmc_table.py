#!/usr/bin/env python
"""Per-kernel mean of rocprofv3 --pmc counter_collection CSVs (one or more passes)."""
import collections
import csv
import sys


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("apex::", "")
            k = (k[5:] if k.startswith("void ") else k).split("(")[0][:70]
            key = (r.get("Dispatch_Id"), r["Counter_Name"])
            acc[k][r["Counter_Name"]].append((key, float(r["Counter_Value"])))
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
    main(sys.argv[1:])
