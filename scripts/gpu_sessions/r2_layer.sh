#!/bin/bash
# round 2: the single-layer row-split measurement on one GPU -- unsharded, and
# through the sharded module at world size 1 (RCCL all-gather inside the captured graph)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r2l_bench 400 python bench.py --no-prefill --no-cpu --steps 16 --warmup 4
step r2l_bench_tp1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --force-shard --no-prefill --no-cpu --steps 16 --warmup 4 --no-extra-weak
