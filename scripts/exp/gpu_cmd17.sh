cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 > gpurun_out/bench_seq2k.log 2>&1; rc=$?; tail -1 gpurun_out/bench_seq2k.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --overlap > gpurun_out/bench_ovl2k.log 2>&1; rc=$?; tail -1 gpurun_out/bench_ovl2k.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
TAG=ovl STEPS=200 BENCH_ARGS=--overlap bash scripts/gpu_profile.sh || exit $?
cd $GRAFT_REPO_ROOT
TAG=seq STEPS=200 bash scripts/gpu_profile.sh
