#!/bin/bash
# round 4, session 10: the product with straight-line two-step waves (K = 4096 WK = 1, K = 8192 WK = 2):
# the whole GPU suite, then the layer chain at P = 1 and the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step r4j_tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r4j_chain1 300 python bench.py --chain-only --chain-shards 1
step r4j_bench 300 python bench.py
echo done
