set -u
cd $GRAFT_REPO_ROOT
for s in "28672 4096" "4096 14336" "8192 28672" "28672 8192" "6144 4096"; do
  echo "=== $s"; timeout -k 10 150 ./scripts/microbench/gemv_micro $s 7 r8 || exit $?
done
