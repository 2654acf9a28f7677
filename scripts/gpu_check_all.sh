#!/bin/bash
# Full check (one gpurun call): the multi-rank IPC tests first (stop-while-credit-blocked
# regression), the whole GPU suite, smoke, a 1-GPU bench, the 3-rank same-device central
# bench (preflight + links), then a kernel + HIP-runtime trace of the 1-GPU step.
# Every GPU step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { echo "== $1 rc=$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_multirank.log 2>&1
rc=$?; step multirank $rc; tail -12 gpurun_out/pytest_multirank.log
[ $rc -ne 0 ] && exit $rc
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread \
  --deselect tests/test_gpu_multirank.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; step suite $rc; tail -6 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; step smoke $rc; tail -2 gpurun_out/smoke.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench1.log 2>&1
rc=$?; step bench1 $rc; grep '^{' gpurun_out/bench1.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 3 --same-device --backend gloo --steps 300 --warmup 20 --capacity 400000 \
  > gpurun_out/bench3_central.log 2>&1
rc=$?; step bench3_central $rc; grep '^{' gpurun_out/bench3_central.log | cut -c1-3000; tail -3 gpurun_out/bench3_central.log | cut -c1-600
[ $rc -ne 0 ] && exit $rc
if [ -z "$SKIP_TRACE" ]; then
O=$R/gpurun_out/trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O -o t \
  -- python3 $R/bench.py --steps 300 --warmup 20 > $O/run.log 2>&1
rc=$?; step trace $rc
fi
exit $rc
