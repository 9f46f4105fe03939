#!/bin/bash
# round 5: greedy pick as partial + final launches -- tests, A/B bench, 8B census
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash scripts/gpu_sessions/r5_s16.sh || exit $?
rm -rf gpurun_out/r5y_*
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5y_an8/trace -- python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r5y_an8.log 2>&1 || exit $?
python3 scripts/decode_anatomy.py gpurun_out/r5y_an8/trace --steps 4 > gpurun_out/r5y_anatomy8.txt 2>&1 || exit $?
rm -rf gpurun_out/r5y_an8/trace
head -14 gpurun_out/r5y_anatomy8.txt | cut -c1-160
echo done
