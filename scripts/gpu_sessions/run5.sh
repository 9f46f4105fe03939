set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/microbench/gemv_micro 4096 4096 > gpurun_out/micro.log 2>&1; rc=$?; echo "micro rc=$rc"; cat gpurun_out/micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-cpu > gpurun_out/bench5.log 2>&1; echo "bench rc=$?"; tail -2 gpurun_out/bench5.log
