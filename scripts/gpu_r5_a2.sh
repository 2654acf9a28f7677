#!/bin/bash
# Round 5 call A2: RNE (1) vs truncation (2) split per launch and whole step, the tree branch
# A/B (per_write_batch vs the round-4 walk), the pinned parameter protocol tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5a2
mkdir -p $O
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_f32_net.py tests/test_gpu_ipc.py \
  > $O/test.log 2>&1; rc=$?; echo "== tests rc=$rc"; grep -E "x6=|passed|failed|Error|published" $O/test.log | head -30
[ $rc -ne 0 ] && exit $rc
for x in 1 2 1 2; do
  timeout -k 10 120 python scripts/bench_f32.py --x6 $x --tile2 > $O/bench_f32_x$x.log 2>&1 || exit $?
  echo "== bench_f32 x6=$x"; grep -v amdgpu.ids $O/bench_f32_x$x.log
done
for rep in 1 2; do
  for v in "1" "2" "1 --tree-walk"; do
    n=$(echo $v | tr ' ' '_')
    timeout -k 10 200 python scripts/ab/x6_bench.py $v --steps 2000 --warmup 50 > $O/bench_${n}_$rep.log 2>&1 || { tail -5 $O/bench_${n}_$rep.log; exit 1; }
    echo "== bench x6=$v rep $rep: $(grep '^{' $O/bench_${n}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
