# sequential and overlapped 1-GPU bench, twice each (run-to-run spread)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 3000 --warmup 50 --no-overlap > gpurun_out/bp_seq$i.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bp_seq$i.log').read().strip().splitlines()[-1]);print('seq',d['value'],d['ms_per_step'])"
timeout -k 10 300 python bench.py --steps 3000 --warmup 50 > gpurun_out/bp_ovl$i.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bp_ovl$i.log').read().strip().splitlines()[-1]);print('ovl',d['value'],d['ms_per_step'])"
done
