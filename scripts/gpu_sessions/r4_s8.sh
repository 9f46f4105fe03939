#!/bin/bash
# round 4, session 8: the early second step with an unconditional issue (OPT 1; the session-2
# variant's conditional issue made hipcc wait for all of step 0 before the table barrier), with
# and without the SGPR-built table (OPT 2); timeline stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for s in "4096 4096" "28672 4096" "6144 4096" "4096 14336" "14336 4096"; do
  set -- $s
  timeout -k 10 240 ./scripts/microbench/gemv_micro $1 $2 7 early > gpurun_out/r4h_early_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median" gpurun_out/r4h_early_$1x$2.log | grep -v floor | cut -c1-100
done
timeout -k 10 200 ./scripts/microbench/gemv_micro 4096 4096 9 stamps > gpurun_out/r4h_stamps.log 2>&1 || exit $?
grep -A3 "OPT" gpurun_out/r4h_stamps.log | head -12
