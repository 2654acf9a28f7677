#!/bin/bash
# Kernel iteration loop (one gpurun call): fp32-net numerics tests (+ EXTRA_TESTS), per-launch
# timing of the learner-shape kernels (scripts/bench_f32.py), a 2000-step bench and, with
# CENTRAL=1, the 3-process central bench on the one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learning.py ${EXTRA_TESTS} -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_kern.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -4 gpurun_out/pytest_kern.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/bench_f32.py > gpurun_out/bench_f32.log 2>&1
rc=$?; echo "== bench_f32 rc=$rc"; cat gpurun_out/bench_f32.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench1.log 2>&1
rc=$?; echo "== bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench1.log | tr '\n' ' '; echo
[ $rc -ne 0 ] && exit $rc
if [ -n "$CENTRAL" ]; then
  timeout -k 10 400 python bench.py --gpus 3 --same-device --backend gloo --steps 300 --warmup 20 --capacity 400000 \
    > gpurun_out/bench3_central.log 2>&1
  rc=$?; echo "== bench3_central rc=$rc"
  grep -o '"value": [0-9.]*\|"links_complete": [a-z]*\|"packets_applied_per_learner_step": [0-9.]*' \
    gpurun_out/bench3_central.log | tr '\n' ' '; echo
fi
exit $rc
