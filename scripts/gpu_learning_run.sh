#!/bin/bash
# Learning evidence on the synthetic game: evaluator tests, random/greedy baselines, then a
# train.py run whose evaluator (eps 0, unclipped rewards) logs the greedy return.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/learn
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_evaluator.py -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/eval_baseline.py > $O/baseline.json 2> $O/baseline.err &&
timeout -k 10 ${TRAIN_SECONDS:-420} python -u -m apex_amd.train --max-step ${MAX_STEP:-100000} --bps_interval 2500 \
  --save_interval 0 --save-path $O/model.pth --no-tb ${TRAIN_ARGS} > $O/train.log 2>&1
