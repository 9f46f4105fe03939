#!/bin/bash
# round 4, session 14: persistent pair grids (QZ_PAIR_PS: 1-8 workgroups per CU, >= 16 the grid) with
# the fused RMSNorm, unsharded gate/up (14336 rows, 1792 blocks) and its shards (7168: 1792 blocks,
# 3584 and 1792: 896 blocks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # M variants
  PAIR_M=$1 PAIR_PS=$2 PAIR_NONORM=0 timeout -k 10 300 python scripts/dev/pair_ps_times.py > gpurun_out/r4n_pair_ps_$1.log 2>&1; local rc=$?
  grep -v amdgpu.ids gpurun_out/r4n_pair_ps_$1.log; [ $rc -eq 0 ] || exit $rc
}
run 14336 0,2,3,4,448,597,640
run 7168 0,2,3,4,448,597,640
run 3584 0,1,2,3,299,448
run 1792 0,1,2,3,299,448
