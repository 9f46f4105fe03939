# multi-token kernel at the per-GPU shard shapes of the driver's weak-scaling runs
# (batch N over TP N): N=8 -> qkv 768x4096, o 4096x512, gate/up 3584x4096, down 4096x1792;
# N=2 -> 3072x4096, 4096x2048, 14336x4096, 4096x7168
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in "768 4096" "4096 512" "3584 4096" "4096 1792" "3072 4096" "4096 2048" "14336 4096" "4096 7168"; do
  timeout -k 10 120 ./scripts/microbench/mt_micro $s || exit $?
done > gpurun_out/mt_shards.txt 2>&1
grep -E "^M=|T=2 TB=2|T=8 TB=8" gpurun_out/mt_shards.txt
