#!/bin/bash
# round 4, session 31: the decode token's kernel census on the round-4 tree (rocprofv3 kernel trace of
# the graph replay; scripts/decode_anatomy.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r4ag_an
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4ag_an/trace -- python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r4ag_an.log 2>&1 || exit $?
python3 scripts/decode_anatomy.py gpurun_out/r4ag_an/trace --steps 4 > gpurun_out/r4ag_anatomy.txt 2>&1 || exit $?
head -40 gpurun_out/r4ag_anatomy.txt | cut -c1-200
