#!/bin/bash
# round 4, session 12: persistent pair workgroups (QZ_PAIR_PS) vs one workgroup per row block
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/dev/pair_ps_times.py > gpurun_out/r4l_pair_ps.log 2>&1; rc=$?
cat gpurun_out/r4l_pair_ps.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
PAIR_M=7168 PAIR_PS=0,1,2,3 timeout -k 10 300 python scripts/dev/pair_ps_times.py > gpurun_out/r4l_pair_ps_7168.log 2>&1; rc=$?
cat gpurun_out/r4l_pair_ps_7168.log | grep -v amdgpu.ids; exit $rc
