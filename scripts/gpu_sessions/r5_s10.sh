#!/bin/bash
# round 5, session 10: the fused-norm whole-row pair as the K = 8192 default (QZ_PAIR_WK1=2) and the
# padded attention v image -- tests, the 70B chain, the 70B decode A/B against QZ_PAIR_WK1=1 on one
# box, and the 8B bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5p_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r5p_tests 400 python -u -m pytest tests/test_gpu_mlp_pair.py tests/test_gpu_prenorm.py tests/test_gpu_mlp_chain.py tests/test_gpu_decode_attention.py -x -q --timeout 120 --timeout-method thread
step r5p_chain70 240 python bench.py --model llama3-70b --chain-only
B70="--model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4"
step r5p_bench70 400 python bench.py $B70
step r5p_bench70_wk1 400 env QZ_PAIR_WK1=1 python bench.py $B70
step r5p_bench8 400 python bench.py --steps 64 --warmup 8
echo done
