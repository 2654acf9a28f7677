#!/bin/bash
# One gpurun call: per-tensor gradient accuracy of one learner step, kernel microbench sweep,
# the 2000-step bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python scripts/diag/grad_check.py > gpurun_out/grad_check.log 2>&1
rc=$?; echo "== grad_check rc=$rc"; cat gpurun_out/grad_check.log | tail -25
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 200 python scripts/bench_f32.py > gpurun_out/bench_f32.log 2>&1
rc=$?; echo "== bench_f32 rc=$rc"; cat gpurun_out/bench_f32.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench1.log 2>&1; rc=$?; echo "== bench rc=$rc"; grep -o "\"value\": [0-9.]*" gpurun_out/bench1.log; exit $rc
