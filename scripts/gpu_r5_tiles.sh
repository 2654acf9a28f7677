#!/bin/bash
# Round 5: forward tile A/B, interleaved on one box: per launch (bench_f32 --tiles) and whole step
# (bench.py --fwd-tile: 0 = 256x64 BK16, 1 = 128x64 (conv3 64x64), 3 = 256x64 BK32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tiles
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  timeout -k 10 150 python scripts/bench_f32.py --tiles 1,3 --only fwd > $O/k_$rep.log 2>&1 || exit $?
  grep -v amdgpu.ids $O/k_$rep.log
done
for rep in 1 2; do
  for t in 0 1 3; do
    timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --fwd-tile $t > $O/b_${t}_$rep.log 2>&1 || exit $?
    echo "fwd_tile=$t rep=$rep $(grep '^{' $O/b_${t}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
