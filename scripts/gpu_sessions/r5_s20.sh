#!/bin/bash
# round 5: counters on the dense lm_head launch (separate passes: kernel trace, FETCH_SIZE, WRITE_SIZE)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
rm -rf gpurun_out/r5lm_*
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r5lm_trace -o run --output-format csv -- python3 scripts/dev/lm_head_only.py > gpurun_out/r5lm_trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r5lm_fetch -o run --output-format csv -- python3 scripts/dev/lm_head_only.py > gpurun_out/r5lm_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5lm_write -o run --output-format csv -- python3 scripts/dev/lm_head_only.py > gpurun_out/r5lm_write.log 2>&1 || exit $?
find gpurun_out/r5lm_* -name "*.csv" | head -20
echo done
