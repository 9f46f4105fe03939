#!/bin/bash
# round 5, session 1: the lean gemv.hip (experiments removed, knobs read once) on the GPU -- the full
# -m gpu suite incl. the new 4- and 8-process one-GPU exchange / row-split tests; the bench line;
# the Llama-3-70B layer chain on 1/2/4/8 ranks' rows and the exchange per call at 4 and 8 processes
# (the config #5 budget)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5a_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r5a_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 420 --timeout-method thread
step r5a_bench 600 python bench.py --steps 32 --warmup 4 --no-cpu
for n in 1 2 4 8; do
  step r5a_chain70_$n 400 python bench.py --model llama3-70b --chain-only --chain-shards $n
done
step r5a_chain8_1 300 python bench.py --chain-only --chain-shards 1
step r5a_xchg4 300 python scripts/exchange_times.py --world 4 --warm
step r5a_xchg8 400 python scripts/exchange_times.py --world 8 --warm
echo done
