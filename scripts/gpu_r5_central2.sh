#!/bin/bash
# Round 5: the central learner's load on one GPU with the final kernels: single-GPU engine vs
# rank 0 with R = 1, 3, 7 emulated links (interleaved), then a kernel trace at R = 7.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R0=$(pwd)
O=$R0/gpurun_out/central6
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 50 > $O/single_$rep.log 2>&1 || exit $?
  echo "single rep=$rep $(grep '^{' $O/single_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  for R in 1 3 7; do
    timeout -k 10 300 python bench.py --emulate-links $R --steps 2000 --warmup 50 > $O/emu${R}_$rep.log 2>&1 || { tail -20 $O/emu${R}_$rep.log; exit 1; }
    echo "emulate R=$R rep=$rep $(grep '^{' $O/emu${R}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['packets_applied_per_learner_step'], d['links_complete'])")"
  done
done
mkdir -p $O/trace7 $O/trace1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace7 -o t -- python3 $R0/bench.py --emulate-links 7 --steps 300 --warmup 20 > $O/trace7/run.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace1 -o t -- python3 $R0/bench.py --emulate-links 1 --steps 300 --warmup 20 > $O/trace1/run.log 2>&1 || exit $?
cd $R0
for R in 1 7; do
  python3 scripts/prof_summary.py $(find $O/trace$R -name "*kernel_trace.csv" | head -1) --marker dqn_heads_bwd --steps 100 > $O/trace$R/summary.md 2>&1
  echo "== trace R=$R"; head -30 $O/trace$R/summary.md
done
