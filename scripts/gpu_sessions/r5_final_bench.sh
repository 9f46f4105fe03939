#!/bin/bash
# round 5, closing: the default bench line on the final tree, plus the FP4 / bf16 / 70B lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5x_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r5x_bench 600 python bench.py
step r5x_bench_fp4 400 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --no-roofline
step r5x_bench_bf16 400 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline
echo done
