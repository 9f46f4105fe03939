# layer ops on the other bench layouts: TP code path at world size 1 (RCCL, sharded heads),
# batch-4 decode; then the full default bench line
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "gpurun_out/$name.log" | cut -c1-260
  [ $rc -eq 0 ] || { tail -5 "gpurun_out/$name.log"; exit $rc; }
}
step bench_force_shard 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --force-shard --no-prefill --no-cpu --no-roofline
step bench_batch4 480 python bench.py --batch 4 --no-prefill --no-cpu --no-roofline
step bench_full2 480 python bench.py
