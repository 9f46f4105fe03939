#!/bin/bash
# round 4, session 6: next-launch prefetch into the Infinity Cache (GEMV chain of rotating copies);
# the layer's Linear4bit chain roofline (bench.py --chain-only) and its kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in "4096 4096" "14336 4096" "4096 14336" "6144 4096"; do
  set -- $s
  timeout -k 10 200 ./scripts/microbench/gemv_micro $1 $2 7 pf > gpurun_out/r4f_pf_$1x$2.log 2>&1 || exit $?
  echo "== $1x$2"; grep -E "median|check" gpurun_out/r4f_pf_$1x$2.log | grep -v floor | cut -c1-110
done
timeout -k 10 300 python bench.py --chain-only > gpurun_out/r4f_chain.log 2>&1 || exit $?
tail -2 gpurun_out/r4f_chain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f_chain_trace -- python3 bench.py --chain-only > gpurun_out/r4f_chain_trace.log 2>&1 || exit $?
echo done
