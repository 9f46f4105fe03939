#!/bin/bash
# round 6: k_gemm16_4d schedules (microbench, no stamps; python sweep vs hipBLASLt) and the
# head-sharded row-split layout on N processes of the one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
(cd scripts/microbench && timeout -k 10 150 ./gemm16_times > ../../gpurun_out/r6_g16_times_4096.txt 2>&1 && \
  timeout -k 10 200 ./gemm16_times 4096 14336 16384 > ../../gpurun_out/r6_g16_times_4096x14336.txt 2>&1 && \
  timeout -k 10 200 ./gemm16_times 14336 4096 16384 > ../../gpurun_out/r6_g16_times_14336x4096.txt 2>&1) || { echo "microbench failed"; exit 1; }
grep -h 'TF/s' gpurun_out/r6_g16_times_*.txt
ROUNDS=11 timeout -k 10 400 python3 -u scripts/gemm16_sched_sweep.py 0,9,11 > gpurun_out/r6_sched_sweep3.txt 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/r6_sched_sweep3.txt; exit 1; }
head -4 gpurun_out/r6_sched_sweep3.txt
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_xgmi_rowsplit.py -x -v --timeout 420 --timeout-method thread -k "heads" > gpurun_out/r6_rowsplit_heads.log 2>&1; tail -8 gpurun_out/r6_rowsplit_heads.log
