#!/bin/bash
# round 3: one-shot protocol times, two processes on one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/exchange_times.py --world 2 > gpurun_out/r3j_times_w2.log 2>&1 || { tail -30 gpurun_out/r3j_times_w2.log; exit 1; }
grep '^{' gpurun_out/r3j_times_w2.log
