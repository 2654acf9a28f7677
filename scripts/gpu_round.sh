#!/bin/bash
# One gpurun call: GPU tests, smoke, 1000-step bench, then a kernel-trace profile of a short
# bench with the per-step Gantt (scripts/prof_timeline.py --dump-step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
OUT="$REPO/gpurun_out/prof_round"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps 100 --warmup 20 > "$OUT/bench_stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -ne 0 ] && exit $rc
T=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
python3 "$REPO/scripts/prof_timeline.py" "$T" --dump-step > "$OUT/timeline.txt" 2>&1
head -8 "$OUT/timeline.txt"
exit 0
