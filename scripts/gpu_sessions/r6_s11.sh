#!/bin/bash
# round 6: counters of the persistent asm GEMM (QZ_GEMM16_SCHED 707) beside hipBLASLt at 4096 x 14336 and 4096^2 (T = 16384)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r6q_*
run() {  # name, shape args, rocprofv3 args...
  local n=$1 shp=$2; shift 2
  timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d gpurun_out/r6q_$n -o run -- python3 scripts/prof_gemm16.py 10 $shp > gpurun_out/r6q_$n.log 2>&1 || { echo "pass $n failed"; tail -5 gpurun_out/r6q_$n.log; exit 1; }
}
export QZ_GEMM16_SCHED=707
for shp in "4096 14336 16384" "4096 4096 16384"; do
  t=s707_$(echo $shp | cut -d' ' -f2)
  run ${t}_trace "$shp" --kernel-trace
  run ${t}_p1 "$shp" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
  run ${t}_p2 "$shp" --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU
  run ${t}_p3 "$shp" --pmc TCC_HIT_sum TCC_MISS_sum
  run ${t}_p4 "$shp" --pmc FETCH_SIZE
  run ${t}_p5 "$shp" --pmc TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TD_BUSY_avr
  python3 scripts/counter_table.py gpurun_out/r6q_${t}_trace gpurun_out/r6q_${t}_p1 gpurun_out/r6q_${t}_p2 gpurun_out/r6q_${t}_p3 gpurun_out/r6q_${t}_p4 gpurun_out/r6q_${t}_p5 > gpurun_out/r6q_${t}_table.txt 2>&1 || { echo "table $t failed"; cat gpurun_out/r6q_${t}_table.txt; exit 1; }
done
echo ok
