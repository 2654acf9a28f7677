#!/bin/bash
# Sample-resident conv2 / conv3 forward (knob 25): numerics test, per-launch timing at the
# learner shapes (3 x 512 samples) and the actor's (256), then bench.py A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/direct
O=gpurun_out/direct
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py -x -q -k "direct or layers or multi_pass" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for k in 25=0 25=1 25=2; do
  timeout -k 10 120 python scripts/bench_f32.py --only fwd --knobs $k > $O/fwd_$k.txt 2>&1 || exit 1
  echo "== $k (B=512 x3)"; cat $O/fwd_$k.txt
  timeout -k 10 120 python scripts/bench_f32.py --only fwd --B 86 --knobs $k > $O/fwd86_$k.txt 2>&1 || exit 1
  echo "== $k (B=86 x3 ~ actor 256)"; grep conv $O/fwd86_$k.txt
done
for k in 25=0 25=1 25=2 25=0 25=1 25=2; do
  APEX_F32_KNOBS=$k timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > $O/bench_$k.log 2>&1 || exit 1
  echo "bench $k: $(grep -o '"value": [0-9.]*' $O/bench_$k.log)"
done
