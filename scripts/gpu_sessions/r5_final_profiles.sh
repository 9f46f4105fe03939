#!/bin/bash
# round 5, closing: rocprofv3 on the bench line's two cited launches as the final tree runs them --
# the 4096^2 roofline GEMV (bench.py --gemv-only) and the dominant decode launch, the gate/up pair
# with the fused norm (bench.py --dominant-only): FETCH / WRITE / SQ passes (one per run) and the
# kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5y_*
pmc() {  # name cmd... (one PMC pass, killed hard at 120 s)
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY"
pmc r5y_gemv_fetch --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5y_gemv_fetch -- python3 bench.py --gemv-only
pmc r5y_gemv_write --pmc WRITE_SIZE --output-format csv -d gpurun_out/r5y_gemv_write -- python3 bench.py --gemv-only
pmc r5y_gemv_trace --kernel-trace --stats --output-format csv -d gpurun_out/r5y_gemv_trace -- python3 bench.py --gemv-only
pmc r5y_dom_fetch --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5y_dom_fetch -- python3 bench.py --dominant-only
pmc r5y_dom_write --pmc WRITE_SIZE --output-format csv -d gpurun_out/r5y_dom_write -- python3 bench.py --dominant-only
pmc r5y_dom_sq --pmc $SQ --output-format csv -d gpurun_out/r5y_dom_sq -- python3 bench.py --dominant-only
pmc r5y_dom_trace --kernel-trace --stats --output-format csv -d gpurun_out/r5y_dom_trace -- python3 bench.py --dominant-only
for d in r5y_gemv_fetch r5y_gemv_write r5y_gemv_trace; do
  python3 scripts/rocprof_summary.py gpurun_out/$d --match k_gemv_4bit --json gpurun_out/$d.json > gpurun_out/$d.summary.txt 2>&1 || exit $?
done
for d in r5y_dom_fetch r5y_dom_write r5y_dom_sq r5y_dom_trace; do
  python3 scripts/rocprof_summary.py gpurun_out/$d --match pair --json gpurun_out/$d.json > gpurun_out/$d.summary.txt 2>&1 || exit $?
done
head -4 gpurun_out/r5y_gemv_fetch.summary.txt gpurun_out/r5y_gemv_trace.summary.txt gpurun_out/r5y_dom_fetch.summary.txt gpurun_out/r5y_dom_trace.summary.txt | cut -c1-220
echo done
