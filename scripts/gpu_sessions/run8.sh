set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in "8192 28672" "28672 4096" "4096 4096"; do
  echo "=== $s"; timeout -k 10 150 ./scripts/microbench/gemv_micro $s 7 ablate || exit $?
done
