# bench: empty-launch + dominant-kernel roofline objects; batched decode (weak-scaling layout) at world 1
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step bench_n1 300 python bench.py --steps 16 --warmup 4 --no-prefill --no-cpu
step bench_b4 300 python bench.py --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline --batch 4
step bench_shard_b4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --force-shard --batch 4 --steps 16 --warmup 4 --no-roofline
step bench_shard_b1_strong 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --force-shard --strong --steps 16 --warmup 4 --no-roofline
