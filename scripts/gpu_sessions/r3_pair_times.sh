#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/dev/pair_times.py > gpurun_out/r3_pair_times.txt 2>&1
rc=$?; cat gpurun_out/r3_pair_times.txt | grep -v amdgpu.ids; exit $rc
