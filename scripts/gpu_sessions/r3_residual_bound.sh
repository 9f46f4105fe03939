#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/dev/residual_upper_bound.py > gpurun_out/r3_residual_bound.txt 2>&1 || { tail -20 gpurun_out/r3_residual_bound.txt; exit 1; }
grep skip gpurun_out/r3_residual_bound.txt
