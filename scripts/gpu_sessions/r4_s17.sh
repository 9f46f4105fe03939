#!/bin/bash
# round 4, session 17: the world-2 one-shot exchange (two processes on the one GPU), sizes ascending
# and descending with every replay's time (the round-3 27.64 us flags outlier at 256 B), world 1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc
}
step r4q_xch2 200 python scripts/exchange_times.py --world 2
step r4q_xch2r 200 python scripts/exchange_times.py --world 2 --reverse
step r4q_xch1 200 python scripts/exchange_times.py --world 1
echo done
