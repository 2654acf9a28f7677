cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 100 --warmup 10 --same-device --backend gloo --capacity 200000 --threshold 20000 > gpurun_out/dp2_ovl.log 2>&1; rc=$?; echo "dp2 overlap rc=$rc"; tail -2 gpurun_out/dp2_ovl.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 100 --warmup 10 --same-device --backend gloo --capacity 200000 --threshold 20000 --topology central > gpurun_out/central2.log 2>&1; rc=$?; echo "central2 rc=$rc"; tail -2 gpurun_out/central2.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
TAG=ovl_f STEPS=300 bash scripts/gpu_profile.sh
cd $GRAFT_REPO_ROOT; TAG=seq_f STEPS=300 BENCH_ARGS=--no-overlap bash scripts/gpu_profile.sh
