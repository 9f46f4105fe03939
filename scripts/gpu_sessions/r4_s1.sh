#!/bin/bash
# round 4, session 1: VALU issue rates of the decode instructions (v_fma_mix_f32, SDWA mov);
# the exact-code GEMV by fp32 codes + v_fma_mix (FMV 1/2) vs the round-3 hi+lo v_dot2c table at
# the decode shapes; SQ counters of the two round-3 product launches (4096^2 CL, gate/up pair +
# RMSNorm + SiLU) and the pair's FETCH/WRITE passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r4a_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
pmc() {  # name cmd... (one PMC pass, killed hard at 120 s)
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r4a_valu 120 ./scripts/microbench/valu_rate
for s in "4096 4096" "28672 4096" "6144 4096" "4096 14336" "14336 4096"; do
  set -- $s
  step r4a_fm_$1x$2 240 ./scripts/microbench/gemv_micro $1 $2 7 fm
done
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY"
pmc r4a_sq_gemv --pmc $SQ --output-format csv -d gpurun_out/r4a_sq_gemv -- python3 bench.py --gemv-only
pmc r4a_sq_dom --pmc $SQ --output-format csv -d gpurun_out/r4a_sq_dom -- python3 bench.py --dominant-only
pmc r4a_fetch_dom --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4a_fetch_dom -- python3 bench.py --dominant-only
pmc r4a_write_dom --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4a_write_dom -- python3 bench.py --dominant-only
pmc r4a_trace_dom --kernel-trace --stats --output-format csv -d gpurun_out/r4a_trace_dom -- python3 bench.py --dominant-only
timeout -k 5 60 rocprofv3 -L > gpurun_out/r4a_counter_list.txt 2>&1 || true
echo done
