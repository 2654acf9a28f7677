#!/bin/bash
# Strided in-block tree walk + small-batch routing: replay / AQL tests, AQL bench, Ape-X bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/treesmall
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_fused_bwd.py tests/test_gpu_aql_engine.py tests/test_gpu_aql.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --algo aql --steps 2000 --warmup 50 > $O/aql.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 > $O/b.log 2>&1
rc=$?
for f in aql b; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
exit $rc
