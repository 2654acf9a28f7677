#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters here).
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/prof_${TAG:-bench}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --steps ${STEPS:-50} --warmup 10 ${BENCH_ARGS:-} > "$OUT/bench_stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 "$OUT/bench_stdout.log"
find "$OUT" -name "*kernel_stats.csv" | head -3
exit $rc
