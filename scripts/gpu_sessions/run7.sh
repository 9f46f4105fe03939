#!/bin/bash
# SQ counter passes on the product GEMV for a large and the headline shape
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
for shp in "8192 28672" "4096 4096"; do
  set -- $shp
  run pmc1_$1x$2 300 rocprofv3 --pmc $C1 --output-format csv -d gpurun_out/pmc1_$1x$2 -- python3 scripts/prof_gemv.py $1 $2 nf4 100
  run pmc2_$1x$2 300 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/pmc2_$1x$2 -- python3 scripts/prof_gemv.py $1 $2 nf4 100
  run trace_$1x$2 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$1x$2 -- python3 scripts/prof_gemv.py $1 $2 nf4 100
done
