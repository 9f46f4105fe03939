#!/bin/bash
# round 4, session 11: issue rates of the fp32 packed ops; exact codes against x widened to fp32
# (FMV 3 = v_fma_f32, FMV 4 = v_pk_fma_f32) vs the hi + lo fp16 code pairs (FMV 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/microbench/valu_rate > gpurun_out/r4k_valu.log 2>&1 || exit $?
grep -E "waves/SIMD (2|4)" gpurun_out/r4k_valu.log | cut -c1-110
for s in "4096 4096" "28672 4096" "6144 4096" "4096 14336" "1024 4096"; do
  set -- $s
  timeout -k 10 240 ./scripts/microbench/gemv_micro $1 $2 7 xf > gpurun_out/r4k_xf_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median|check" gpurun_out/r4k_xf_$1x$2.log | grep -v floor | cut -c1-100
done
