#!/bin/bash
# Forced-DP (1-rank) step with the direct RCCL communicator vs torch.distributed, and
# the single-process step, 1000 timed steps each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d['config'].get('dp_comm'))"; }
for c in ${COMMS:-rccl torch}; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29519 bench.py --force-dp --comm $c --steps ${STEPS:-1000} --warmup 50 ${BENCH_ARGS:-} > gpurun_out/comm_$c.log 2>&1 || { tail -30 gpurun_out/comm_$c.log; exit 1; }
  summ gpurun_out/comm_$c.log "forced-dp comm=$c"
done
timeout -k 10 200 python bench.py --steps ${STEPS:-1000} --warmup 50 ${BENCH_ARGS:-} > gpurun_out/comm_single.log 2>&1 || { tail -20 gpurun_out/comm_single.log; exit 1; }
summ gpurun_out/comm_single.log "single"
