#!/bin/bash
# kernel trace of the self-launched 3-rank central bench on one GPU (rank 0 learner + replay,
# ranks 1-2 actors over HIP IPC): every rank writes its own trace (the tool library is inherited)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd); O=$R/gpurun_out/central_prof; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 $R/bench.py --gpus 3 --same-device \
  --backend gloo --topology central --steps 200 --warmup 20 --capacity 300000 --threshold 20000 --launch-timeout 300 > $O/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep '^{' $O/bench.log | cut -c1-300; find $O -name "*kernel_trace.csv" | head; exit $rc
