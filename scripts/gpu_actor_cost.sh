#!/bin/bash
# What the local actor costs the learner, one box: overlapped engine (default), serial engine,
# a 32-env actor, and the central learner with one emulated link (no actor on the GPU).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/actor_cost
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 150 python -u bench.py --steps 2000 --warmup 50 "$@" > $O/$tag.log 2>&1 || exit $?; echo "$tag $(tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("actor_frames_per_sec"))')"; }
run overlap
run serial --no-overlap
run envs32 --envs 32
run emu1 --emulate-links 1
run overlap2
