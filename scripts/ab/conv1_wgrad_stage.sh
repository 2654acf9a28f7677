#!/bin/bash
# conv1 weight gradient staging fix (plane addresses resolved once, loads all in flight): numerics
# tests, per-launch timing, bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/c1w
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32_net.py tests/test_gpu_learning.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/bench_f32.py --only bwd > $O/bwd.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/bench_f32.py --only conv1_wgrad > $O/c1w.txt 2>&1 || exit 1
cat $O/bwd.txt $O/c1w.txt | grep -v amdgpu.ids
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > $O/bench_$r.log 2>&1 || exit 1
  echo "bench: $(grep -o '"value": [0-9.]*' $O/bench_$r.log)"
done
