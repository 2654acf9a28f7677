#!/bin/bash
# kernel-trace Gantt of the bench step with --target-ahead 1 (and 0 for reference)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
for t in 1 0; do
  OUT="$REPO/gpurun_out/ta_prof$t"; mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
    python3 "$REPO/bench.py" --steps 100 --warmup 20 --target-ahead $t > "$OUT/bench_stdout.log" 2>&1
  rc=$?; echo "rocprof ahead=$t rc=$rc"; [ $rc -ne 0 ] && exit $rc
  T=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
  python3 "$REPO/scripts/prof_timeline.py" "$T" --dump-step > "$OUT/timeline.txt" 2>&1
  head -6 "$OUT/timeline.txt"
  rm -f "$T"
done
exit 0
