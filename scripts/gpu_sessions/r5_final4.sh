#!/bin/bash
# round 5, closing (after the sliced norm launch): whole GPU suite + smoke, the bench lines (8B default,
# FP4, bf16, 70B on one GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
}
bash scripts/gpu_sessions/r5_final_tests.sh || exit $?
rm -rf gpurun_out/r5q4_*
step r5q4_bench 600 python bench.py
step r5q4_bench_fp4 400 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --no-roofline
step r5q4_bench_bf16 400 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline
step r5q4_bench70 600 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline
echo done
