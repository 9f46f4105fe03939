#!/bin/bash
# round 4, session 32: the normed q/k/v launch with its second K-step issued before the prologue
# barriers (QZ_GROUPED_EARLY), A/B twice on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
QKV_VARIANTS=0:0:0:0,0:0:0:1,0:0:0:0,0:0:0:1 timeout -k 10 300 python scripts/dev/qkv_ps_times.py > gpurun_out/r4ah_qkv_early.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4ah_qkv_early.log; [ $rc -eq 0 ] || exit $rc
QKV_MS=14336,14336 QKV_COPIES=8 QKV_VARIANTS=0:0:0:0,0:0:0:1 timeout -k 10 300 python scripts/dev/qkv_ps_times.py > gpurun_out/r4ah_gateup_early.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4ah_gateup_early.log; exit $rc
