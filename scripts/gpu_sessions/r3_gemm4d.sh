#!/bin/bash
# round 3: 4-wave LDS-DMA 16-bit GEMM (k_gemm16_4d) vs the 8-phase plain kernel, gemm_micro
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
make -C scripts/microbench gemm_micro > gpurun_out/r3_gemm4d_build.log 2>&1 || { tail -20 gpurun_out/r3_gemm4d_build.log; exit 1; }
for s in "4096 4096" "14336 4096" "4096 14336"; do
  timeout -k 10 120 ./scripts/microbench/gemm_micro $s >> gpurun_out/r3_gemm4d.txt 2>&1 || { tail -20 gpurun_out/r3_gemm4d.txt; exit 1; }
done
cat gpurun_out/r3_gemm4d.txt
