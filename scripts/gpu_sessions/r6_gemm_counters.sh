#!/bin/bash
# round 6: counters of qz_gemm_16bit (k_gemm16_4d) beside hipBLASLt's kernel at config #4 (4096^2, T = 16384)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r6g_*
run() {  # name, rocprofv3 args...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d gpurun_out/r6g_$n -o run -- python3 scripts/prof_gemm16.py 10 > gpurun_out/r6g_$n.log 2>&1 || { echo "pass $n failed"; tail -5 gpurun_out/r6g_$n.log; exit 1; }
}
run trace --kernel-trace
run p1 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run p2 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU
run p3 --pmc TCC_HIT_sum TCC_MISS_sum
run p4 --pmc FETCH_SIZE
python3 scripts/counter_table.py gpurun_out/r6g_trace gpurun_out/r6g_p1 gpurun_out/r6g_p2 gpurun_out/r6g_p3 gpurun_out/r6g_p4 | tee gpurun_out/r6g_table.txt
