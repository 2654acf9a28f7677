cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_fused_net.py tests/test_gpu_overlap.py tests/test_gpu_learner.py -q -rf -x > gpurun_out/pytest_multi.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_multi.log
if [ $rc -ne 0 ]; then tail -80 gpurun_out/pytest_multi.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench_seq_m.log 2>&1; rc=$?; tail -1 gpurun_out/bench_seq_m.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --overlap > gpurun_out/bench_ovl_m.log 2>&1; rc=$?; tail -1 gpurun_out/bench_ovl_m.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
TAG=ovl_m STEPS=200 BENCH_ARGS=--overlap bash scripts/gpu_profile.sh
