#!/bin/bash
# Round 5: the overlapped actor graph confined to a CU subset (hipExtStreamCreateWithCUMask) vs
# every CU -- whole-step A/B, interleaved on one box, then a kernel trace of the best setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/actor_cus
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for c in 0 32 64 128; do
    timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --actor-cus $c > $O/b_${c}_$rep.log 2>&1 || { tail -20 $O/b_${c}_$rep.log; exit 1; }
    echo "actor_cus=$c rep=$rep $(grep '^{' $O/b_${c}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
