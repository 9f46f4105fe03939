#!/bin/bash
# round 3: persistent streaming GEMV (K = 4096) vs the production full-step kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for s in "28672 4096" "14336 4096" "6144 4096" "4096 4096"; do
  echo "=== $s"; timeout -k 10 200 ./scripts/microbench/gemv_micro $s 7 stream || exit $?
done
