#!/bin/bash
# round 4, session 7: the world-2 one-shot exchange outlier (sizes ascending and descending, every
# replay's time); the layer chain on one rank's rows at P = 1/2/4/8; the whole GPU suite; the default
# bench line
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
step r4g_xch2 200 python scripts/exchange_times.py --world 2
step r4g_xch2r 200 python scripts/exchange_times.py --world 2 --reverse
step r4g_xch1 200 python scripts/exchange_times.py --world 1
for P in 1 2 4 8; do step r4g_chain$P 300 python bench.py --chain-only --chain-shards $P; done
step r4g_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r4g_bench 700 python bench.py
echo done
