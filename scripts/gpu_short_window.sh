#!/bin/bash
# The driver's short window (--steps 20 --warmup 5) against a long run, one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/short
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 150 python -u bench.py "$@" > $O/$tag.log 2>&1 || exit $?; echo "$tag $(tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
run s20a --steps 20 --warmup 5
run long --steps 2000 --warmup 50
run s20b --steps 20 --warmup 5
run s20c --steps 20 --warmup 50
run s200 --steps 200 --warmup 5
