#!/bin/bash
# PMC passes over the fp32 network kernels (eager launches of scripts/bench_f32.py), then the table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_pmc_f32.sh || exit $?
cd $R && python3 scripts/pmc_table.py --summary $(find gpurun_out/pmc_f32 -name "*counter_collection.csv") > gpurun_out/pmc_f32/table.md 2>&1
rc=$?; cat gpurun_out/pmc_f32/table.md; exit $rc
