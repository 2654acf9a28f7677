#!/usr/bin/env python
"""Align a rocprofv3 HIP-runtime trace with its kernel trace (``--kernel-trace
--hip-runtime-trace``): for a window of consecutive hipGraphLaunch calls, the host
interval of each call next to the GPU interval of the kernels it launched (kernels carry
the launching call's correlation id), the idle gap on each queue before the graph's first
kernel, and one step's kernel Gantt.  Used for VERDICT r3 item 4 (the step-start hole)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("api")
    ap.add_argument("kernels")
    ap.add_argument("--first", type=int, default=200, help="index of the first hipGraphLaunch in the window")
    ap.add_argument("--n", type=int, default=16)
    a = ap.parse_args()
    api = list(csv.DictReader(open(a.api)))
    ks = sorted(csv.DictReader(open(a.kernels)), key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in ks:
        by.setdefault(r["Correlation_Id"], []).append(r)
    gls = sorted((x for x in api if x["Function"] == "hipGraphLaunch"), key=lambda x: int(x["Start_Timestamp"]))
    win = gls[a.first:a.first + a.n]
    t0 = int(win[0]["Start_Timestamp"])
    last_end = {}
    print("hipGraphLaunch host interval (us)  |  its kernels on the GPU (us)  |  queue idle before (us)  first kernel")
    for x in win:
        hs, he = int(x["Start_Timestamp"]) - t0, int(x["End_Timestamp"]) - t0
        kk = by.get(x["Correlation_Id"], [])
        if not kk:
            print(f"{hs / 1e3:9.1f} - {he / 1e3:9.1f}   (no kernels)")
            continue
        q = kk[0]["Queue_Id"]
        gs = min(int(r["Start_Timestamp"]) for r in kk) - t0
        ge = max(int(r["End_Timestamp"]) for r in kk) - t0
        gap = gs - last_end[q] if q in last_end else float("nan")
        last_end[q] = ge
        print(f"{hs / 1e3:9.1f} - {he / 1e3:9.1f}   |  {gs / 1e3:9.1f} - {ge / 1e3:9.1f}  n={len(kk):2d} q{q}"
              f"  |  {gap / 1e3:7.1f}  {kk[0]['Kernel_Name'][:48]}")
    x, y = win[2], win[3]
    kk = sorted(by.get(x["Correlation_Id"], []) + by.get(y["Correlation_Id"], []),
                key=lambda r: int(r["Start_Timestamp"]))
    if kk:
        s0 = int(kk[0]["Start_Timestamp"])
        print("\none step (two consecutive graph launches): start  dur  queue  kernel")
        for r in kk:
            s, e = int(r["Start_Timestamp"]) - s0, int(r["End_Timestamp"]) - s0
            print(f"{s / 1e3:8.1f} {(e - s) / 1e3:6.1f}  q{r['Queue_Id']:>2}  {r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
