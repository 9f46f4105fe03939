#!/bin/bash
# round 5, closing: the whole GPU suite and smoke() on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5z_*
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5z_gpu_tests.log 2>&1
rc=$?; echo "== gpu tests rc=$rc"; tail -3 gpurun_out/r5z_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5z_smoke.log 2>&1
rc=$?; echo "== smoke rc=$rc"; tail -2 gpurun_out/r5z_smoke.log; exit $rc
