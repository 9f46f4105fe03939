set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in "4096 4096" "1024 4096" "14336 4096" "4096 14336" "8192 8192" "1024 8192" "28672 8192" "8192 28672"; do
  echo "=== $s"; timeout -k 10 120 ./scripts/microbench/gemv_micro $s 7 sweep || exit $?
done
