#!/bin/bash
# round 4, session 23: the persistent exact-code pair on the 256-B-entry table (QZ_PAIR_WT: 64 KiB,
# conflict-free, one v_perm per address) at 2 / 3 workgroups per CU vs the 16-copy table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 14336 7168; do
  PAIR_M=$m PAIR_PS=0,3,2,1002,1003,1001 PAIR_NONORM=0 timeout -k 10 300 python scripts/dev/pair_ps_times.py > gpurun_out/r4x_pair_wt_$m.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/r4x_pair_wt_$m.log; [ $rc -eq 0 ] || exit $rc
done
