#!/bin/bash
# round 2 final: smoke, whole GPU suite, default bench line, config #3 (FP4, no DQ) and
# config #5 (Llama-3-70B, one GPU) decode lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r2f_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r2f_pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r2f_bench 480 python bench.py
step r2f_bench_fp4 300 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --steps 32 --warmup 4
step r2f_bench_70b 480 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline
