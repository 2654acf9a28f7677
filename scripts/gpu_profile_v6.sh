#!/bin/bash
# Steady-state profiles of the current default: overlap (kernel stats + step Gantt) and the
# sequential step (--no-overlap, per-kernel table), plus an un-profiled 2000-step bench and
# the forced-DP bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/bench.log | cut -c1-300
STEPS=2000 bash scripts/ab/gpu_forcedp.sh 2>&1 | grep -v rc= || exit 1
cd /tmp && export TMPDIR=/tmp
for mode in overlap seq; do
  OUT="$REPO/gpurun_out/prof_v6_$mode"; mkdir -p "$OUT"
  ARGS=""; [ $mode = seq ] && ARGS="--no-overlap"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$REPO/bench.py" --steps 300 --warmup 30 $ARGS > "$OUT/bench_stdout.log" 2>&1 || exit 1
  T=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
  python3 "$REPO/scripts/prof_timeline.py" "$T" --steps 250 --dump-step > "$OUT/timeline.txt" 2>&1
  python3 "$REPO/scripts/prof_summary.py" "$T" --marker dqn_heads_bwd --steps 250 > "$OUT/summary.txt" 2>&1
  head -5 "$OUT/timeline.txt"
done
exit 0
