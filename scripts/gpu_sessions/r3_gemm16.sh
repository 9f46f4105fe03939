#!/bin/bash
# round 3: qz_gemm_16bit on the 4-wave LDS-DMA kernel: edge tests, then the route sweep vs hipBLASLt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -k gemm16 -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_gemm16_tests.log 2>&1 || { tail -40 gpurun_out/r3_gemm16_tests.log; exit 1; }
tail -3 gpurun_out/r3_gemm16_tests.log
timeout -k 10 400 python -u scripts/prefill_route_sweep.py ${1:-4096,16384} > gpurun_out/r3_gemm16_sweep.txt 2>&1 || { tail -20 gpurun_out/r3_gemm16_sweep.txt; exit 1; }
grep -v "^{\"" gpurun_out/r3_gemm16_sweep.txt | cut -c1-400
