#!/bin/bash
# round 4, session 20: rocprofv3 on the dominant decode launch as it now runs (the persistent gate/up
# pair with the fused norm): SQ counters, FETCH / WRITE passes, kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r4u_*
pmc() {  # name cmd... (one PMC pass, killed hard at 120 s)
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY"
pmc r4u_sq_dom --pmc $SQ --output-format csv -d gpurun_out/r4u_sq_dom -- python3 bench.py --dominant-only
pmc r4u_fetch_dom --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4u_fetch_dom -- python3 bench.py --dominant-only
pmc r4u_write_dom --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4u_write_dom -- python3 bench.py --dominant-only
pmc r4u_trace_dom --kernel-trace --stats --output-format csv -d gpurun_out/r4u_trace_dom -- python3 bench.py --dominant-only
for d in r4u_sq_dom r4u_fetch_dom r4u_write_dom r4u_trace_dom; do
  python3 scripts/rocprof_summary.py gpurun_out/$d --match pair --json gpurun_out/$d.json > gpurun_out/$d.summary.txt 2>&1 || exit $?
  head -30 gpurun_out/$d.summary.txt | cut -c1-250
done
echo done
