set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for s in "8192 28672" "28672 4096" "4096 4096"; do
  echo "=== $s"; timeout -k 10 150 ./scripts/microbench/gemv_micro $s 7 ablate || exit $?
done > gpurun_out/ablate2.log 2>&1
