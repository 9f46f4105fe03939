#!/bin/bash
# round 4, session 13: persistent pair workgroups by row blocks per workgroup (QZ_PAIR_PS) at the
# unsharded gate/up (14336 rows) and its row shards at N = 2 / 4 / 8 (7168 / 3584 / 1792 rows)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 14336 7168 3584 1792; do
  PAIR_M=$m timeout -k 10 300 python scripts/dev/pair_ps_times.py > gpurun_out/r4m_pair_ps_$m.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/r4m_pair_ps_$m.log; [ $rc -eq 0 ] || exit $rc
done
