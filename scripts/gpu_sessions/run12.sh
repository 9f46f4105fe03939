#!/bin/bash
# Round-1 evidence: full bench line, then rocprofv3 kernel trace + PMC passes (gemv roofline) and a decode trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; tail -1 gpurun_out/bench_full.log; [ $rc -eq 0 ] || exit $rc
DECODE_CMD="python3 bench.py --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline" bash scripts/gpu_profile.sh
