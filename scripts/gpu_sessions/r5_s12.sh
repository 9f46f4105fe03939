#!/bin/bash
# round 5, session 12: q/k/v projections + decode attention in one launch (csrc/qkv_attn.hip) --
# parity tests (fused vs the two launches, the refactored standalone attention), then the 8B bench
# with and without it on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5r_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r5r_tests 300 python -u -m pytest tests/test_gpu_qkv_attention.py tests/test_gpu_decode_attention.py -x -q --timeout 120 --timeout-method thread
step r5r_bench8 300 python bench.py --steps 64 --warmup 8 --no-prefill --no-cpu --no-roofline
step r5r_bench8_off 300 python bench.py --steps 64 --warmup 8 --no-prefill --no-cpu --no-roofline --no-qkv-attention
step r5r_bench8_2 300 python bench.py --steps 64 --warmup 8 --no-prefill --no-cpu --no-roofline
echo done
