#!/bin/bash
# round 4, session 34: the other configs' bench lines on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step r4aj_fp4 400 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --steps 32 --warmup 4
step r4aj_bf16 400 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
step r4aj_70b 600 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
echo done
