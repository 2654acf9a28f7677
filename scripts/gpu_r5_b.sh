#!/bin/bash
# Round 5 call B: PMC of the X6 GEMM kernels, the actor-CU-mask A/B, the bf16 re-bench, and a
# kernel trace of the default step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/r5b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_f32_net.py tests/test_gpu_learner.py \
  > $O/test.log 2>&1; rc=$?; echo "== tests rc=$rc"; grep -E "conv2_fwd|passed|failed|Error" $O/test.log | head
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > $O/bench_$i.log 2>&1 || exit $?
  echo "== bench $i $(grep '^{' $O/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 120 python scripts/bench_f32.py --tile2 > $O/bench_f32.log 2>&1 || exit $?
grep -v amdgpu.ids $O/bench_f32.log
bash scripts/gpu_pmc_r4.sh > $O/pmc.log 2>&1; rc=$?; echo "== pmc rc=$rc"; tail -14 $O/pmc.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for c in 0 32 64; do
    timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --actor-cus $c > $O/cus_${c}_$rep.log 2>&1 || { tail -20 $O/cus_${c}_$rep.log; exit 1; }
    echo "actor_cus=$c rep=$rep $(grep '^{' $O/cus_${c}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --dtype bf16 > $O/bf16.log 2>&1 || exit $?
echo "== bf16 $(grep '^{' $O/bf16.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
mkdir -p $O/trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 $R/bench.py --steps 300 --warmup 20 > $O/trace/run.log 2>&1
rc=$?; echo "== trace rc=$rc"
cd $R && python3 scripts/prof_summary.py $(find $O/trace -name "*kernel_trace.csv" | head -1) --marker dqn_heads_bwd --steps 100 > $O/trace/summary.md 2>&1; head -40 $O/trace/summary.md
exit $rc
