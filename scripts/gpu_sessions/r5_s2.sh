#!/bin/bash
# round 5, session 2: the persistent MLP half-layer (csrc/chain.hip) -- its bit-identity tests, the
# pair tests on the explicit knob setter, the layer chain with the chain kernel vs three launches,
# the bench line, and a kernel trace of the chain
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5b_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step r5b_chain_tests 300 python -u -m pytest tests/test_gpu_mlp_chain.py -x -v --timeout 120 --timeout-method thread
step r5b_pair_tests 300 python -u -m pytest tests/test_gpu_mlp_pair.py tests/test_gpu_prenorm.py -x -q --timeout 120 --timeout-method thread
step r5b_chain8 300 python bench.py --chain-only
step r5b_chain8_3l 300 python bench.py --chain-only --chain-three-launch
step r5b_bench 600 python bench.py --steps 32 --warmup 4 --no-cpu --no-prefill
step r5b_bench_nochain 600 python bench.py --steps 32 --warmup 4 --no-cpu --no-prefill --no-roofline --no-mlp-chain --no-extra-codes
step r5b_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5b_trace -- python3 bench.py --chain-only
echo done
