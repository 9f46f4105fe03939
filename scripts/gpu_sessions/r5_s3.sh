#!/bin/bash
# round 5, session 3: the chain with act staged in LDS -- tests, chain per layer vs three launches,
# stage timeline stamps (diagnostic build), bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5c_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-500
  [ $rc -eq 0 ] || exit $rc
}
step r5c_chain_tests 300 python -u -m pytest tests/test_gpu_mlp_chain.py -x -q --timeout 120 --timeout-method thread
step r5c_stamps 300 python scripts/dev/chain_stamps.py
step r5c_chain8 300 python bench.py --chain-only
step r5c_chain8_3l 300 python bench.py --chain-only --chain-three-launch
step r5c_chain70 300 python bench.py --model llama3-70b --chain-only
step r5c_stamps70 300 python scripts/dev/chain_stamps.py --model llama3-70b --samples 2
echo done
