#!/bin/bash
# 8-wave gate/up pair launch with the fused pre-norm: pair tests (bit-identity), pair launch
# times at 4 vs 8 waves, same-box bench A/B, then the attention phase ablation
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3d_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -3 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r3d_pair_tests 300 python -u -m pytest tests/test_gpu_mlp_pair.py tests/test_gpu_prenorm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
QZ_PAIR_WAVES=4 step r3d_pair_times_w4 200 python scripts/dev/pair_times.py
QZ_PAIR_WAVES=8 step r3d_pair_times_w8 200 python scripts/dev/pair_times.py
QZ_PAIR_WAVES=8 step r3d_bench_w8 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
QZ_PAIR_WAVES=4 step r3d_bench_w4 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
QZ_PAIR_WAVES=8 step r3d_bench_w8b 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
step r3d_attn_abl 240 python scripts/dev/attn_ablation.py
