#!/bin/bash
# One gpurun call: IPC primitive + multi-rank central tests, then the self-launched
# 3-rank central bench on one GPU (rank 0 learner, ranks 1-2 actors, HIP IPC transport).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_multirank.py -x -v -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_ipc.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_ipc.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 3 --same-device --backend gloo --topology central --steps 300 --warmup 20 \
  --capacity 300000 --threshold 20000 --launch-timeout 240 > gpurun_out/bench_central_ipc3.log 2>&1
rc=$?; echo "bench central rc=$rc"; grep '^{' gpurun_out/bench_central_ipc3.log | cut -c1-1500; tail -3 gpurun_out/bench_central_ipc3.log | cut -c1-500
exit $rc
