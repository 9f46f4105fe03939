#!/bin/bash
# round 4, session 33: the final-tree check (smoke, GPU suite, bench), then the persistent wide-table pair
# at R = 2 vs 4 rows per wave (QZ_PAIR_R, read once per process)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_sessions/r4_s29.sh || exit $?
for r in 2 4; do
  QZ_PAIR_R=$r PAIR_M=14336 PAIR_PS=0,1002 PAIR_NONORM=0 timeout -k 10 300 python scripts/dev/pair_ps_times.py > gpurun_out/r4ai_pair_r$r.log 2>&1; rc=$?
  echo "== R=$r"; grep -v amdgpu.ids gpurun_out/r4ai_pair_r$r.log; [ $rc -eq 0 ] || exit $rc
done
