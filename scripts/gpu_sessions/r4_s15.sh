#!/bin/bash
# round 4, session 15: the persistent pair grid sweep (r4_s14), then the product with the default
# persistent grid for the normed pair: whole GPU suite, layer chain, bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_sessions/r4_s14.sh || exit $?
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-800
  [ $rc -eq 0 ] || exit $rc
}
step r4o_tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r4o_chain1 300 python bench.py --chain-only --chain-shards 1
step r4o_bench 300 python bench.py
echo done
