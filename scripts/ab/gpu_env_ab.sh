#!/bin/bash
# A/B of HIP runtime graph-launch knobs on the single-process and forced-DP benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
i=0
for envs in "${@}"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --steps 1000 --warmup 50 ${BENCH_ARGS:-} > gpurun_out/env_single_$i.log 2>&1 || { tail -20 gpurun_out/env_single_$i.log; exit 1; }
  summ gpurun_out/env_single_$i.log "single [$envs]"
  env $envs timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29519 bench.py --force-dp --steps 1000 --warmup 50 ${BENCH_ARGS:-} > gpurun_out/env_fdp_$i.log 2>&1 || { tail -20 gpurun_out/env_fdp_$i.log; exit 1; }
  summ gpurun_out/env_fdp_$i.log "forced-dp [$envs]"
done
