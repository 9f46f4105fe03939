#!/bin/bash
# fused decode attention: its tests, the model-level tests that now run it, the bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
step r3at_tests 400 python -u -m pytest tests/test_gpu_decode_attention.py tests/test_gpu_layer_ops.py tests/test_gpu_prenorm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step r3at_bench 400 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
