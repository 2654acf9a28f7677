# A/B of bench variants: BENCH_VARIANTS="label:args|label:args" (each run twice)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
IFS='|' read -ra VARS <<< "$BENCH_VARIANTS"
for i in 1 2; do
for v in "${VARS[@]}"; do
  label=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python bench.py --steps 3000 --warmup 50 $a > gpurun_out/ab_${label}_$i.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ab_${label}_$i.log').read().strip().splitlines()[-1]);print('$label',d['value'],d['ms_per_step'],'host',d.get('host_enqueue_ms_per_step'))"
done
done
