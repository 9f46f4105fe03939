#!/bin/bash
# round 6: the hand-ordered asm step of k_gemm16_4d (S 65): bit-identity, then times against 0 / 9 and hipBLASLt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gemm16_sched.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_sched_tests4.log 2>&1 || { tail -30 gpurun_out/r6_sched_tests4.log; exit 1; }
tail -1 gpurun_out/r6_sched_tests4.log
(cd scripts/microbench && timeout -k 10 150 ./gemm16_times > ../../gpurun_out/r6_g16_times3_4096.txt 2>&1 && \
  timeout -k 10 200 ./gemm16_times 4096 14336 16384 > ../../gpurun_out/r6_g16_times3_4096x14336.txt 2>&1 && \
  timeout -k 10 150 ./gemm16_stamps > ../../gpurun_out/r6_g16_stamps3_4096.txt 2>&1) || { echo "microbench failed"; exit 1; }
grep -h 'TF/s' gpurun_out/r6_g16_times3_*.txt | cut -c1-40
grep -h 'S=65\|S=9 \|S=0 ' gpurun_out/r6_g16_stamps3_4096.txt
ROUNDS=9 timeout -k 10 500 python3 -u scripts/gemm16_sched_sweep.py 0,9,65 > gpurun_out/r6_sched_sweep5.txt 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/r6_sched_sweep5.txt; exit 1; }
head -4 gpurun_out/r6_sched_sweep5.txt
