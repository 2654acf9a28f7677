#!/bin/bash
# Full-step A/B of f32_kernels.hip: current vs the round-4 version before the conv1 rework
# (scripts/ab/old/f32_kernels_f3b0dea.hip), rebuilt on the box; bench A, B, A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
F=ape-x_amd/ops/csrc/f32_kernels.hip
cp $F gpurun_out/ab/cur.hip
b() { timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/ab/b.log 2>&1 || return $?;
      echo "$1: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"; }
rb() { timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/ab/build.log 2>&1; }
b cur || exit $?
cp scripts/ab/old/f32_kernels_f3b0dea.hip $F && rb || exit $?
b old || exit $?
cp gpurun_out/ab/cur.hip $F && rb || exit $?
b cur || exit $?
cp scripts/ab/old/f32_kernels_f3b0dea.hip $F && rb || exit $?
b old || exit $?
cp gpurun_out/ab/cur.hip $F
