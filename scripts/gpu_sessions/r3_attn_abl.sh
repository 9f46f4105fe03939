#!/bin/bash
# price the phases of the decode attention kernel (QZ_ATTN_ABL builds, back-to-back and graph)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python scripts/dev/attn_ablation.py > gpurun_out/r3c_attn_abl.txt 2>&1
rc=$?; echo "== abl rc=$rc"; cat gpurun_out/r3c_attn_abl.txt | tail -12
exit $rc
