#!/bin/bash
# Full-step A/B of f32_kernels.hip: current vs an alternative kernel file ALT (default: the
# double-buffered conv1 version, `git show 70b5b2a:ape-x_amd/ops/csrc/f32_kernels.hip > alt.hip`),
# rebuilt on the box; bench A, B, A, B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
F=ape-x_amd/ops/csrc/f32_kernels.hip
cp $F gpurun_out/ab/cur.hip
b() { timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/ab/b.log 2>&1 || return $?;
      echo "$1: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"; }
rb() { timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/ab/build.log 2>&1; }
b cur || exit $?
cp ${ALT:-scripts/ab/alt_f32_kernels.hip} $F && rb || exit $?
b old || exit $?
cp gpurun_out/ab/cur.hip $F && rb || exit $?
b cur || exit $?
cp ${ALT:-scripts/ab/alt_f32_kernels.hip} $F && rb || exit $?
b old || exit $?
cp gpurun_out/ab/cur.hip $F
