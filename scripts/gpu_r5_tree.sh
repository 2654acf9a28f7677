#!/bin/bash
# Round 5: learner tree branch on per_write_batch -- tree / learner / overlap tests, bench x2, PMC of the X6 GEMMs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -s -x -v --timeout 120 --timeout-method thread tests/test_gpu_replay.py \
  tests/test_gpu_fused_bwd.py tests/test_gpu_learner.py tests/test_gpu_overlap.py tests/test_gpu_learning.py tests/test_gpu_ipc.py tests/test_gpu_multirank.py tests/test_gpu_aql_engine.py tests/test_gpu_central_aql.py tests/test_gpu_f32_net.py \
  > gpurun_out/r5_tree_test.log 2>&1; rc=$?; echo "== tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r5_tree_test.log | tail -15
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > gpurun_out/r5_bench_tree$i.log 2>&1 || exit $?
  echo "== bench $i"; grep '^{' gpurun_out/r5_bench_tree$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
bash scripts/gpu_pmc_r4.sh
bash scripts/gpu_prof_bench.sh _r5 && python3 scripts/prof_summary.py $(find gpurun_out/prof_bench_r5 -name "*kernel_trace.csv" | head -1) --marker dqn_heads_bwd --steps 100 > gpurun_out/prof_bench_r5/summary.md 2>&1; tail -40 gpurun_out/prof_bench_r5/summary.md
