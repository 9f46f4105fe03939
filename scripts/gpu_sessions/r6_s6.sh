#!/bin/bash
# round 6: k_gemm16_4d with the SIMD-parity staggered schedule (S 25 / 27) against 0 / 9 / 11 and hipBLASLt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm16_sched.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_sched_tests3.log 2>&1 || { tail -20 gpurun_out/r6_sched_tests3.log; exit 1; }
tail -1 gpurun_out/r6_sched_tests3.log
(cd scripts/microbench && timeout -k 10 150 ./gemm16_times > ../../gpurun_out/r6_g16_times2_4096.txt 2>&1 && \
  timeout -k 10 200 ./gemm16_times 4096 14336 16384 > ../../gpurun_out/r6_g16_times2_4096x14336.txt 2>&1) || { echo "microbench failed"; exit 1; }
grep -h 'TF/s' gpurun_out/r6_g16_times2_*.txt | cut -c1-40
ROUNDS=11 timeout -k 10 500 python3 -u scripts/gemm16_sched_sweep.py 0,9,25,27 > gpurun_out/r6_sched_sweep4.txt 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/r6_sched_sweep4.txt; exit 1; }
head -4 gpurun_out/r6_sched_sweep4.txt
