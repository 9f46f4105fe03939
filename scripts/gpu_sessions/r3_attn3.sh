#!/bin/bash
# decode attention with one query head per workgroup: attention tests, phase ablation, bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3e_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -3 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r3e_attn_tests 300 python -u -m pytest tests/test_gpu_decode_attention.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step r3e_attn_abl 240 python scripts/dev/attn_ablation.py
step r3e_bench 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
step r3e_bench2 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
