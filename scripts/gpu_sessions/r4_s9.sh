#!/bin/bash
# round 4, session 9: straight-line two-step GEMV waves (OPT 8: step 2 issued right after the
# barrier, not after all of step 1 arrived); timeline stamps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for s in "4096 4096" "28672 4096" "6144 4096" "14336 4096" "1024 4096"; do
  set -- $s
  timeout -k 10 240 ./scripts/microbench/gemv_micro $1 $2 7 two > gpurun_out/r4i_two_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median|check" gpurun_out/r4i_two_$1x$2.log | grep -v floor | cut -c1-100
done
timeout -k 10 200 ./scripts/microbench/gemv_micro 4096 4096 9 stamps > gpurun_out/r4i_stamps.log 2>&1 || exit $?
grep -A4 "OPT 8\|(product)" gpurun_out/r4i_stamps.log | head -14
