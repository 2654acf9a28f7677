#!/bin/bash
# One gpurun call: GPU suite, 1-GPU bench, then the self-launched 2-rank same-device gloo
# bench (bench.py --gpus 2 without torch.distributed.run).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log | cut -c1-600
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 1000 --warmup 50 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench1.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 2 --same-device --backend gloo --steps 50 --warmup 5 --capacity 200000 \
  --launch-timeout 300 > gpurun_out/bench2_gloo.log 2>&1
rc=$?; echo "bench2 gloo rc=$rc"; tail -4 gpurun_out/bench2_gloo.log | cut -c1-1500
exit $rc
