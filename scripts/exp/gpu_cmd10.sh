cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 2 --topology central --backend gloo --same-device --steps 60 --warmup 5 --capacity 200000 --threshold 20000 --envs 128 > gpurun_out/central2.log 2>&1; rc=$?; echo "central rc=$rc"; tail -3 gpurun_out/central2.log | cut -c1-600
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29712 bench.py --gpus 2 --backend gloo --same-device --steps 60 --warmup 5 --capacity 200000 --threshold 20000 --envs 128 > gpurun_out/sharded2.log 2>&1; rc=$?; echo "sharded rc=$rc"; tail -3 gpurun_out/sharded2.log | cut -c1-600
exit $rc
