#!/bin/bash
# round 5, session 4: Llama-3-70B gate/up through the pair launch at K = 8192 (whole rows per wave,
# persistent workgroups, norm + SiLU fused) -- tests, the 70B layer chain, and the 70B decode A/B on
# one box against the round-4 form (QZ_PAIR_WK1=0: grouped gate/up + separate norm and SiLU launches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5d_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
[ "${1:-}" = bench ] && rm -f gpurun_out/r5d_tests.log
[ "${1:-}" = bench ] || step r5d_tests 400 python -u -m pytest tests/test_gpu_mlp_pair.py tests/test_gpu_prenorm.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
[ "${1:-}" = bench ] || step r5d_chain70 300 python bench.py --model llama3-70b --chain-only
[ "${1:-}" = bench ] || step r5d_chain70_old 300 env QZ_PAIR_WK1=0 python bench.py --model llama3-70b --chain-only
[ "${1:-}" = bench ] || { echo done; exit 0; }
step r5d_bench70 540 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
step r5d_bench70_old 540 env QZ_PAIR_WK1=0 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
echo done
