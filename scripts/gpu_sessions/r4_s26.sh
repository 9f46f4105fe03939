#!/bin/bash
# round 4, session 26: 8-wave workgroups on the 256-B-entry exact-code table vs the product geometry at
# the o_proj (4096^2), down_proj (4096 x 14336), q/k/v (6144 x 4096) and 70B shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for s in "4096 4096" "4096 14336" "6144 4096" "8192 28672" "1024 4096"; do
  set -- $s
  timeout -k 10 240 ./scripts/microbench/gemv_micro $1 $2 7 nw8 > gpurun_out/r4aa_nw8_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median|check" gpurun_out/r4aa_nw8_$1x$2.log | grep -v floor | cut -c1-100
done
