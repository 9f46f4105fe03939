#!/bin/bash
# residual adds in the GEMV epilogues: tests, then bench with / without
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3rs
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/r3rs/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/r3rs/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
step tests 400 python -u -m pytest tests/test_gpu_mlp_pair.py tests/test_gpu_residual.py tests/test_gpu_decode_attention.py tests/test_gpu_layer_ops.py tests/test_gpu_prenorm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_res 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
step bench_nores 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes --no-residual
step bench_res2 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
