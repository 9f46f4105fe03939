#!/bin/bash
# round 6 (closing): kernel trace + MFMA-busy counters of qz_gemm_16bit's default schedule (963, k_gemm16_4q W-first)
# beside hipBLASLt's kernel at config #4's three shapes (T = 16384, randn fp16)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r6z_*
run() {  # name, shape args, rocprofv3 args...
  local n=$1 shp=$2; shift 2
  timeout -s KILL 120 rocprofv3 "$@" --output-format csv -d gpurun_out/r6z_$n -o run -- python3 scripts/prof_gemm16.py 10 $shp > gpurun_out/r6z_$n.log 2>&1 || { echo "pass $n failed"; tail -5 gpurun_out/r6z_$n.log; exit 1; }
}
for shp in "4096 4096 16384" "14336 4096 16384" "4096 14336 16384"; do
  t=$(echo $shp | cut -d' ' -f1)x$(echo $shp | cut -d' ' -f2)
  run ${t}_trace "$shp" --kernel-trace --stats
  run ${t}_p1 "$shp" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
  python3 scripts/counter_table.py gpurun_out/r6z_${t}_trace gpurun_out/r6z_${t}_p1 > gpurun_out/r6z_${t}_table.txt 2>&1 || { echo "table $t failed"; exit 1; }
done
echo ok
