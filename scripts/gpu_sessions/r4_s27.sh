#!/bin/bash
# round 4, session 27: 8-wave wide-table launches for K >= 14336 exact-code GEMVs: parity tests, 8B and
# 70B bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r4ab_tests 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_residual.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r4ab_70b 600 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
step r4ab_bench 300 python bench.py
echo done
