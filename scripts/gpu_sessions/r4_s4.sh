#!/bin/bash
# round 4, session 4: MFMA-product GEMV with lane-masked x loads; the product kernel with x
# staged in LDS (XL) under exact codes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for s in "4096 4096" "14336 4096" "28672 4096" "6144 4096"; do
  set -- $s
  timeout -k 10 200 ./scripts/microbench/gemv_micro $1 $2 7 dg > gpurun_out/r4e_dg_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median|check" gpurun_out/r4e_dg_$1x$2.log | grep -v floor | cut -c1-110
done
