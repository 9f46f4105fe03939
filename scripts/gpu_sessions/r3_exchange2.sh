#!/bin/bash
# round 3: tagged-granule one-shot all-gather: two-process test, tp1 bench path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi_exchange.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3i_exchange.log 2>&1 || { tail -40 gpurun_out/r3i_exchange.log; exit 1; }
tail -2 gpurun_out/r3i_exchange.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-shard --steps 32 --warmup 4 --no-prefill --no-cpu --no-extra-weak --no-extra-codes > gpurun_out/r3i_tp1.log 2>&1 || { tail -30 gpurun_out/r3i_tp1.log; exit 1; }
grep -o '"rowsplit_layer".*' gpurun_out/r3i_tp1.log; grep -o '"value": [0-9.]*' gpurun_out/r3i_tp1.log | head -1; grep -o '"exchange": "[^"]*"' gpurun_out/r3i_tp1.log
