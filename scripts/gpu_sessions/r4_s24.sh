#!/bin/bash
# round 4, session 24: default = persistent exact-code pair on the 256-B-entry table at 2 per CU:
# the shard sizes, pair tests, full GPU suite, chain, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 3584 1792; do
  PAIR_M=$m PAIR_PS=0,3,2,1002 PAIR_NONORM=0 timeout -k 10 300 python scripts/dev/pair_ps_times.py > gpurun_out/r4y_pair_wt_$m.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/r4y_pair_wt_$m.log; [ $rc -eq 0 ] || exit $rc
done
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step r4y_tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r4y_chain1 300 python bench.py --chain-only --chain-shards 1
step r4y_bench 300 python bench.py
echo done
