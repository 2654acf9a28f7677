"""Instruction mix of each kernel's hottest basic block in a gfx950 assembly listing.

Usage: python scripts/diag/isa_loop_mix.py <file.s> [name-filter]

For every kernel the block with the most MFMAs is taken as its main loop; the script prints
the block's MFMA, VALU (vector ALU, MFMA excluded), LDS, vector-memory and scalar counts and
VALU per MFMA -- the static form of the PMC 'VALU / MFMA' column (profiles/r5_fp32_pmc.md),
available without a GPU.  Generate the listing with
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip --cuda-device-only -S <src.hip> -o <file.s>
"""
from __future__ import annotations

import re
import subprocess
import sys


def blocks(lines):
    kern, blk, body = None, None, []
    for ln in lines:
        m = re.match(r"^([_A-Za-z][\w.$]*):", ln)
        if m and not ln.startswith("."):
            name = m.group(1)
            if not name.startswith(".L"):
                if blk is not None:
                    yield kern, blk, body
                kern, blk, body = name, name, []
                continue
        m = re.match(r"^(\.LBB[\w_]+):", ln)
        if m:
            if blk is not None:
                yield kern, blk, body
            blk, body = m.group(1), []
            continue
        s = ln.strip()
        if s and not s.startswith((".", ";", "//")):
            body.append(s.split()[0])
    if blk is not None:
        yield kern, blk, body


def mix(body):
    c = {"mfma": 0, "valu": 0, "lds": 0, "vmem": 0, "salu": 0}
    for op in body:
        if "mfma" in op:
            c["mfma"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    best = {}
    with open(path) as f:
        for kern, blk, body in blocks(f.read().splitlines()):
            c = mix(body)
            if kern not in best or c["mfma"] > best[kern][1]["mfma"]:
                best[kern] = (blk, c)
    names = list(best)
    for name, dn in zip(names, demangle(names)):
        if filt and filt not in dn:
            continue
        blk, c = best[name]
        if not c["mfma"]:
            continue
        print(f"{dn[:90]:90s} mfma {c['mfma']:4d} valu {c['valu']:5d} ({c['valu'] / c['mfma']:5.2f}/mfma) "
              f"lds {c['lds']:4d} vmem {c['vmem']:4d} salu {c['salu']:4d}")


if __name__ == "__main__":
    main()
