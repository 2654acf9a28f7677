#!/bin/bash
# DP split: FC1 weight gradient in place (APEX_FC1_DP_INPLACE=1, default) vs sliced + finalized
# before the FC1 all-reduce (=0); forced-DP 1-rank bench, interleaved; DP tests at the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fc1dp
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp_rccl.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  APEX_FC1_DP_INPLACE=$v timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 2954$v bench.py --force-dp --steps 3000 --warmup 50 > $O/b$v.log 2>&1 || exit 1
  echo "forced-dp inplace=$v: $(grep -h '^{' $O/b$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
