#!/bin/bash
# round 3: price of the GEMV prologue's global loads (timing-only variant)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for s in "4096 4096" "6144 4096" "28672 4096" "4096 14336"; do
  echo "=== $s"; timeout -k 10 200 ./scripts/microbench/gemv_micro $s 7 nopro || exit $?
done
