# multi-token kernel: waves per workgroup (W = 4 / 8 (product) / 16) at the weak-scaling shard shapes
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in "768 4096" "3584 4096" "4096 1792" "4096 512" "3072 4096" "14336 4096" "4096 7168" "4096 4096"; do
  timeout -k 10 120 ./scripts/microbench/mt_micro $s waves || exit $?
done > gpurun_out/mt_waves.txt 2>&1
cat gpurun_out/mt_waves.txt
