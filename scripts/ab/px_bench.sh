#!/bin/bash
# One gpurun call: learner parity with the 8-term px forward, fp32 bench with px 0 / 1 / 2
# (knob 19: off / 6 / 8 term products), then a kernel-trace profile of the px 2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPO=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
APEX_F32_KNOBS="19=2" timeout -k 10 300 python -u -m pytest tests/test_gpu_learning.py -k fp32 -x -v -s --timeout 240 --timeout-method thread > gpurun_out/learning_parity_px8.txt 2>&1
rc=$?; echo "parity px8 rc=$rc"; grep "^0 \|^199 \|passed\|failed" gpurun_out/learning_parity_px8.txt
for px in 0 1 2 0 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --px $px > gpurun_out/bench_px$px.log 2>&1
  rc=$?; echo "bench px=$px rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench_px$px.log | tr '\n' ' '; echo
  [ $rc -ne 0 ] && exit $rc
done
OUT="$REPO/gpurun_out/prof_px"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps 100 --warmup 20 --px 2 > "$OUT/bench_stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -ne 0 ] && exit $rc
T=$(find "$OUT" -name "*kernel_stats.csv" | head -1); head -25 "$T" | cut -d, -f1-4 | cut -c1-150
exit 0
