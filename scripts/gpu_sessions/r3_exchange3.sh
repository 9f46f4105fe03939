#!/bin/bash
# round 3: both one-shot protocols -- two-process test, per-call times by payload (world 1, world 2 on one GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi_exchange.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r3j_exchange.log 2>&1 || { tail -40 gpurun_out/r3j_exchange.log; exit 1; }
tail -1 gpurun_out/r3j_exchange.log
timeout -k 10 300 python scripts/exchange_times.py --world 1 > gpurun_out/r3j_times_w1.log 2>&1 || { tail -30 gpurun_out/r3j_times_w1.log; exit 1; }
grep '^{' gpurun_out/r3j_times_w1.log
timeout -k 10 300 python scripts/exchange_times.py --world 2 > gpurun_out/r3j_times_w2.log 2>&1 || { tail -30 gpurun_out/r3j_times_w2.log; exit 1; }
grep '^{' gpurun_out/r3j_times_w2.log
