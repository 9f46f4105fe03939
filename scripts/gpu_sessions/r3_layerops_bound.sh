#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/dev/layer_op_upper_bound.py > gpurun_out/r3_layerops_bound.txt 2>&1 || { tail -20 gpurun_out/r3_layerops_bound.txt; exit 1; }
cat gpurun_out/r3_layerops_bound.txt | grep skip
