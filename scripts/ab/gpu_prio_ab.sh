#!/bin/bash
# A/B of the high-priority stream choice, single-process and forced-DP (1-rank RCCL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d.get('stream_probe'))"; }
for p in ${PRIOS:-none}; do
  timeout -k 10 200 python bench.py --steps ${STEPS:-1000} --warmup 50 --streams $p > gpurun_out/ab_single_$p.log 2>&1 || { tail -20 gpurun_out/ab_single_$p.log; exit 1; }
  summ gpurun_out/ab_single_$p.log "single prio=$p"
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29519 bench.py --force-dp --steps ${STEPS:-1000} --warmup 50 --streams $p > gpurun_out/ab_fdp_$p.log 2>&1 || { tail -20 gpurun_out/ab_fdp_$p.log; exit 1; }
  summ gpurun_out/ab_fdp_$p.log "forced-dp prio=$p"
done
