#!/bin/bash
# Async central topology rehearsal on ONE GPU (gloo, host-staged links): the single-rank
# engine (same learner config) vs rank 0 learner + 1 and 2 actor ranks.  Every step has its
# own time limit; steps chained with &&.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/central
mkdir -p $O
cd $R
COMMON="--steps ${STEPS:-2000} --warmup 50 --capacity 262144 --threshold 20000 --envs 256"
timeout -k 10 200 python -u bench.py $COMMON > $O/single.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --topology central --backend gloo --same-device $COMMON > $O/central2.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
  --master-port 29532 bench.py --gpus 3 --topology central --backend gloo --same-device $COMMON > $O/central3.log 2>&1
rc=$?
for f in single central2 central3; do echo "== $f"; grep '^{' $O/$f.log | cut -c1-700; done
exit $rc
