#!/bin/bash
# round 3: one-shot IPC all-gather (two processes on the one GPU), the tp1 row-split bench path
# with the one-shot exchange, then the whole GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3d_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step r3d_exchange 300 python -u -m pytest tests/test_gpu_xgmi_exchange.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step r3d_tp1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-shard --steps 32 --warmup 4 --no-prefill --no-cpu --no-extra-weak
step r3d_pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
