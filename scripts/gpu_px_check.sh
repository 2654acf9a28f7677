#!/bin/bash
# One gpurun call: px numerics tests, then fp32 bench without / with the pre-split forward,
# then a kernel-trace profile of the px bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_px.py -x -v -s -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_px.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed|px errors" gpurun_out/pytest_px.log | tail -12
[ $rc -ne 0 ] && exit $rc
# learner parity (HIP fp32 learner vs torch fp32 / fp64 on one sampled stream, 200 steps), plain and px
timeout -k 10 300 python -u -m pytest tests/test_gpu_learning.py -k fp32 -x -v -s --timeout 240 --timeout-method thread > gpurun_out/learning_parity_fp32.txt 2>&1
rc=$?; echo "parity fp32 rc=$rc"; tail -2 gpurun_out/learning_parity_fp32.txt
[ $rc -ne 0 ] && exit $rc
APEX_F32_KNOBS="19=1" timeout -k 10 300 python -u -m pytest tests/test_gpu_learning.py -k fp32 -x -v -s --timeout 240 --timeout-method thread > gpurun_out/learning_parity_px.txt 2>&1
rc=$?; echo "parity px rc=$rc"; tail -2 gpurun_out/learning_parity_px.txt
[ $rc -ne 0 ] && exit $rc
for px in 0 1; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --px $px > gpurun_out/bench_px$px.log 2>&1
  rc=$?; echo "bench px=$px rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench_px$px.log | tr '\n' ' '; echo
  [ $rc -ne 0 ] && exit $rc
done
OUT="$REPO/gpurun_out/prof_px"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps 100 --warmup 20 --px 1 > "$OUT/bench_stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -ne 0 ] && exit $rc
T=$(find "$OUT" -name "*kernel_stats.csv" | head -1); head -25 "$T" | cut -d, -f1-4 | cut -c1-150
exit 0
