#!/bin/bash
# round 3: scalar-prologue GEMV A/B (microbench), timeline stamps at 4096^2, one-shot exchange without fences
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in "4096 4096" "6144 4096" "28672 4096" "4096 14336" "8192 8192"; do
  echo "=== $s"; timeout -k 10 200 ./scripts/microbench/gemv_micro $s 7 sp || exit $?
done
timeout -k 10 200 ./scripts/microbench/gemv_micro 4096 4096 1 stamps > gpurun_out/r3e_stamps.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi_exchange.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3e_exchange.log 2>&1 || { tail -30 gpurun_out/r3e_exchange.log; exit 1; }
tail -2 gpurun_out/r3e_exchange.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-shard --steps 32 --warmup 4 --no-prefill --no-cpu --no-extra-weak --no-extra-codes > gpurun_out/r3e_tp1.log 2>&1 || exit $?
grep -o '"rowsplit_layer".*' gpurun_out/r3e_tp1.log; grep -o '"value": [0-9.]*' gpurun_out/r3e_tp1.log | head -1
