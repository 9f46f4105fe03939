#!/bin/bash
# rocprofv3 passes (kernel trace, then PMC passes on their own) -> gpurun_out/prof_*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
P="${PROFILE_CMD:-python3 bench.py --gemv-only}"
run prof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -- $P
run prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -- $P
run prof_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -- $P
if [ -n "${DECODE_CMD:-}" ]; then
  run prof_decode 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_decode -- $DECODE_CMD
fi
