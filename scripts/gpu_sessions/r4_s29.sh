#!/bin/bash
# round 4, session 29: the current tree end to end: smoke, the whole GPU suite, the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r4ad_smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step r4ad_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r4ad_bench 300 python bench.py
echo done
