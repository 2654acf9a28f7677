#!/bin/bash
# Effective shader clock per kernel (GRBM_GUI_ACTIVE / duration): the learner's kernels alone
# (bench_f32, eager) vs inside the overlapped engine step (bench.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/clock
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o iso -- python3 $GRAFT_REPO_ROOT/scripts/bench_f32.py --iters 3 --graph 0 > $O/iso.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o step -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 10 --no-graphs > $O/step.log 2>&1
