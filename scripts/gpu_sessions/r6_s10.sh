#!/bin/bash
# round 6: the persistent asm-step GEMM k_gemm16_4q (QZ_GEMM16_SCHED 579 = 512|67, 707 = 512|195): bit-identity,
# microbench, randn and uniform sweeps against hipBLASLt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm16_sched.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_sched_tests6.log 2>&1 || { tail -30 gpurun_out/r6_sched_tests6.log; exit 1; }
tail -1 gpurun_out/r6_sched_tests6.log
(cd scripts/microbench && timeout -k 10 150 ./gemm16_times > ../../gpurun_out/r6_g16_times5_4096.txt 2>&1 && \
  timeout -k 10 200 ./gemm16_times 4096 14336 16384 > ../../gpurun_out/r6_g16_times5_4096x14336.txt 2>&1) || { echo "microbench failed"; exit 1; }
grep -h 'TF/s' gpurun_out/r6_g16_times5_*.txt | cut -c1-40
ROUNDS=7 timeout -k 10 400 python3 -u scripts/gemm16_sched_sweep.py 0,195,579,707 > gpurun_out/r6_sched_sweep8.txt 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/r6_sched_sweep8.txt; exit 1; }
head -4 gpurun_out/r6_sched_sweep8.txt
DATA=uniform ROUNDS=5 timeout -k 10 400 python3 -u scripts/gemm16_sched_sweep.py 0,195,707 > gpurun_out/r6_sched_sweep8_uniform.txt 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/r6_sched_sweep8_uniform.txt; exit 1; }
head -4 gpurun_out/r6_sched_sweep8_uniform.txt
