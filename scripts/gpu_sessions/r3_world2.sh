#!/bin/bash
# round 3: row-split at world 2 on the real kernels with the one-shot exchange (two processes on the one GPU),
# the exchange test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xgmi_rowsplit.py tests/test_gpu_xgmi_exchange.py -m gpu -x -v -s --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/r3l_world2.log 2>&1 || { tail -60 gpurun_out/r3l_world2.log; exit 1; }
tail -4 gpurun_out/r3l_world2.log
