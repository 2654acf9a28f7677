#!/bin/bash
# Single-GPU measurement of the data-parallel step: real RCCL collectives in a 1-rank
# group (--force-dp) vs the single-process step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29519 bench.py --force-dp --steps ${STEPS:-1000} --warmup 50 ${BENCH_ARGS:-} > gpurun_out/forcedp.log 2>&1
rc=$?; echo "force-dp rc=$rc"; grep '^{' gpurun_out/forcedp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('forced-dp', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
[ $rc -ne 0 ] && { tail -20 gpurun_out/forcedp.log; exit $rc; }
timeout -k 10 300 python bench.py --steps ${STEPS:-1000} --warmup 50 ${BENCH_ARGS:-} > gpurun_out/single.log 2>&1
rc=$?; echo "single rc=$rc"; grep '^{' gpurun_out/single.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('single', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
exit $rc
