#!/bin/bash
# round 4, session 28: A/B on one box, QZ_GEMV_WIDE8 = 0 / 1 (8-wave wide-table down_proj): the layer
# chain, the 8B bench (no prefill / cpu), the 70B bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
for rep in 1 2; do
for w in 0 1; do
  export QZ_GEMV_WIDE8=$w
  step r4ac_chain_w${w}_$rep 300 python bench.py --chain-only --chain-shards 1
  step r4ac_8b_w${w}_$rep 300 python bench.py --no-prefill --no-cpu --no-roofline --steps 64 --warmup 8
done
done
for w in 0 1; do
  export QZ_GEMV_WIDE8=$w
  step r4ac_70b_w$w 600 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
done
echo done
