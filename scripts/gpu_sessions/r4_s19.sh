#!/bin/bash
# round 4, session 19: a ring of 3 / 4 step buffers (OPT 16 / 32) for waves owning exactly NSW steps:
# Llama-3-8B down_proj (4096 x 14336, 7 steps), Llama-3-70B down_proj (8192 x 28672, 14 steps);
# then the world-2 exchange tests with the warm-up graph
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in "4096 14336" "8192 28672" "14336 14336"; do
  set -- $s
  timeout -k 10 240 ./scripts/microbench/gemv_micro $1 $2 7 ring > gpurun_out/r4t_ring_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median|check" gpurun_out/r4t_ring_$1x$2.log | cut -c1-100
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi_exchange.py tests/test_gpu_xgmi_rowsplit.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4t_xgmi_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4t_xgmi_tests.log; exit $rc
