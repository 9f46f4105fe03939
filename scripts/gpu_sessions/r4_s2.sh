#!/bin/bash
# round 4, session 2: the GEMV prologue -- second K-step issued before the table barrier (OPT 1),
# byte table built from SGPR planes instead of a global load (OPT 2) -- at the decode shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for s in "4096 4096" "28672 4096" "6144 4096" "4096 14336" "14336 4096" "8192 8192"; do
  set -- $s
  timeout -k 10 240 ./scripts/microbench/gemv_micro $1 $2 7 early > gpurun_out/r4b_early_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median|check" gpurun_out/r4b_early_$1x$2.log | cut -c1-120
done
