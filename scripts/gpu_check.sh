#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> short bench.  Each GPU step has
# its own time limit; a crash/timeout (rc not in {0,1}) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -q --maxfail=40"}
BENCH_ARGS=${BENCH_ARGS:-"--steps 16 --warmup 4"}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 600 python -m pytest $PYTEST_ARGS -p no:cacheprovider
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 280 python bench.py $BENCH_ARGS
