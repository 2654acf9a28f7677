#!/bin/bash
# Refresh the secondary bench records: bf16 opt-in, AQL engine, 10M filled replay.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rec2
mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --dtype bf16 > $O/bf16.log 2>&1 &&
timeout -k 10 300 python -u bench.py --algo aql --steps 2000 --warmup 50 > $O/aql.log 2>&1 &&
timeout -k 10 500 python -u bench.py --capacity 10000000 --fill --steps 1000 --warmup 50 > $O/fill10m.log 2>&1
rc=$?
for f in bf16 aql fill10m; do echo "== $f"; grep '^{' $O/$f.log | cut -c1-600; done
exit $rc
