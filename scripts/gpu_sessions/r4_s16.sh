#!/bin/bash
# round 4, session 16: default persistent pair grid = 3 workgroups per CU: pair/prenorm/sharded GPU
# tests, the chain at P = 1 / 2 / 4 / 8 (one rank's rows), bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
step r4p_tests 400 python -u -m pytest tests/test_gpu_mlp_pair.py tests/test_gpu_prenorm.py tests/test_gpu_xgmi_rowsplit.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for P in 1 2 4 8; do step r4p_chain$P 300 python bench.py --chain-only --chain-shards $P; done
step r4p_bench 300 python bench.py
echo done
