#!/bin/bash
# Round 5: the central learner's load on one GPU -- emulated links R = 1, 3, 7 (tests + bench),
# an actor rank's unpaced frames/s at E = 256 / 1024 / 4096, the 3-process same-GPU central run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/central5
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/central5
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_central_emulated.py \
  > $O/test.log 2>&1; rc=$?; echo "== tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/test.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > $O/single.log 2>&1 || exit $?
echo "== single"; grep '^{' $O/single.log | cut -c1-300
for R in 1 3 7; do
  timeout -k 10 300 python bench.py --emulate-links $R --steps 2000 --warmup 50 > $O/emu$R.log 2>&1 || { echo "emu $R failed"; tail -20 $O/emu$R.log; exit 1; }
  echo "== emulate $R"; grep '^{' $O/emu$R.log | cut -c1-900
done
timeout -k 10 300 python bench.py --actor-only 256,1024,4096 --steps 500 --warmup 20 > $O/actor_only.log 2>&1 || { tail -20 $O/actor_only.log; exit 1; }
echo "== actor only"; grep '^{' $O/actor_only.log
timeout -k 10 400 python bench.py --gpus 3 --same-device --backend gloo --steps 300 --warmup 20 --capacity 400000 \
  > $O/bench3_central.log 2>&1; rc=$?; echo "== bench3_central rc=$rc"; grep '^{' $O/bench3_central.log | cut -c1-1500
exit $rc
