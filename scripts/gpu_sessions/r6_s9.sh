#!/bin/bash
# round 6: counters of the asm-step schedules (QZ_GEMM16_SCHED 195, 65) beside hipBLASLt at 4096^2 and 4096 x 14336
# (T = 16384), then the uniform-operand sweep (clock-independent gap)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r6h_*
run() {  # name, shape args, rocprofv3 args...
  local n=$1 shp=$2; shift 2
  timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d gpurun_out/r6h_$n -o run -- python3 scripts/prof_gemm16.py 10 $shp > gpurun_out/r6h_$n.log 2>&1 || { echo "pass $n failed"; tail -5 gpurun_out/r6h_$n.log; exit 1; }
}
for sc in 195 65; do
  export QZ_GEMM16_SCHED=$sc
  for shp in "4096 4096 16384" "4096 14336 16384"; do
    t=s${sc}_$(echo $shp | cut -d' ' -f2)
    run ${t}_trace "$shp" --kernel-trace
    run ${t}_p1 "$shp" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
    run ${t}_p2 "$shp" --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU
    python3 scripts/counter_table.py gpurun_out/r6h_${t}_trace gpurun_out/r6h_${t}_p1 gpurun_out/r6h_${t}_p2 > gpurun_out/r6h_${t}_table.txt 2>&1 || { echo "table $t failed"; cat gpurun_out/r6h_${t}_table.txt; exit 1; }
    echo "== $t"; cat gpurun_out/r6h_${t}_table.txt
  done
done
unset QZ_GEMM16_SCHED
DATA=uniform ROUNDS=7 timeout -k 10 400 python3 -u scripts/gemm16_sched_sweep.py 0,65,195 > gpurun_out/r6_sched_sweep7_uniform.txt 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/r6_sched_sweep7_uniform.txt; exit 1; }
head -4 gpurun_out/r6_sched_sweep7_uniform.txt
