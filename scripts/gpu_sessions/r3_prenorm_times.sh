#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/dev/prenorm_times.py > gpurun_out/r3p_times.txt 2>&1 || { tail -20 gpurun_out/r3p_times.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r3p_times.txt
timeout -k 10 480 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes --no-prenorm > gpurun_out/r3p_70b_noprenorm.log 2>&1 || { tail -5 gpurun_out/r3p_70b_noprenorm.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3p_70b_noprenorm.log
