cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_overlap.py tests/test_gpu_train_cli.py tests/test_gpu_learner.py tests/test_gpu_actor.py -q -rf -x > gpurun_out/pytest_overlap.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_overlap.log
if [ $rc -ne 0 ]; then tail -80 gpurun_out/pytest_overlap.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_seq.log 2>&1; rc=$?; tail -1 gpurun_out/bench_seq.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --overlap > gpurun_out/bench_ovl.log 2>&1; rc=$?; tail -1 gpurun_out/bench_ovl.log | cut -c1-200
exit $rc
