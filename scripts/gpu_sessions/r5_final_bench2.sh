#!/bin/bash
# round 5, closing (after the decode glue): default bench line, FP4 / bf16 lines, 70B on one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5f_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step r5f_bench 600 python bench.py
step r5f_bench_fp4 400 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --no-roofline
step r5f_bench_bf16 400 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline
step r5f_bench70 600 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline
echo done
