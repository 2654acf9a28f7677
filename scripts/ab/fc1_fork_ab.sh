#!/bin/bash
# FC1 finalize forked vs in line: fp32 learner numerics tests, then interleaved 1-GPU benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_learning.py tests/test_gpu_learner.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/ab/t.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -2 gpurun_out/ab/t.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --fc1-fork $v > gpurun_out/ab/b.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ab/b.log; exit $rc; }
    echo "fc1_fork=$v: $(grep -o '"value": [0-9.]*' gpurun_out/ab/b.log)"
  done
done
