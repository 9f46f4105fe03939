#!/bin/bash
# round 3: exact-code table geometry (conflict-free 64 KiB table at 8 waves per workgroup)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for s in "4096 4096" "6144 4096" "28672 4096" "4096 14336" "14336 4096"; do
  echo "=== $s"; timeout -k 10 200 ./scripts/microbench/gemv_micro $s 7 wt8 || exit $?
done
