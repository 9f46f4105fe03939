#!/bin/bash
# round 4, session 30: rocprofv3 on the 4096^2 roofline launch as it now runs (two-step waves): FETCH /
# WRITE passes and the kernel trace, for the bench line's roofline.traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r4af_*
pmc() {  # name cmd... (one PMC pass, killed hard at 120 s)
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pmc r4af_fetch --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4af_fetch -- python3 bench.py --gemv-only
pmc r4af_write --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4af_write -- python3 bench.py --gemv-only
pmc r4af_trace --kernel-trace --stats --output-format csv -d gpurun_out/r4af_trace -- python3 bench.py --gemv-only
for d in r4af_fetch r4af_write r4af_trace; do
  python3 scripts/rocprof_summary.py gpurun_out/$d --match k_gemv_4bit --json gpurun_out/$d.json > gpurun_out/$d.summary.txt 2>&1 || exit $?
  head -12 gpurun_out/$d.summary.txt | cut -c1-250
done
