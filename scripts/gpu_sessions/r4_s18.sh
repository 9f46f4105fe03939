#!/bin/bash
# round 4, session 18: is the slow first flags graph at world 2 a first-graph effect? granules timed
# first; a throwaway flags graph first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "--granules-first" "--warm" ""; do
  n=r4r_xch2$(echo "$v" | tr -d ' -')
  timeout -k 10 200 python scripts/exchange_times.py --world 2 $v > gpurun_out/$n.log 2>&1; rc=$?
  echo "== $n rc=$rc"; grep '"world"' gpurun_out/$n.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['first'], d['warm_graph'], {k:(v['flags'], v['granules']) for k,v in d['us_per_call'].items()})"
  [ $rc -eq 0 ] || exit $rc
done
