#!/bin/bash
# round 4, session 25: persistent q/k/v grouped launch with the fused norm (QZ_GROUPED_PS / _R / _WT)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prenorm.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k persistent > gpurun_out/r4z_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4z_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/dev/qkv_ps_times.py > gpurun_out/r4z_qkv_ps.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4z_qkv_ps.log; exit $rc
