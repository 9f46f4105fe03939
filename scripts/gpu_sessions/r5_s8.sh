#!/bin/bash
# round 5, session 8: the whole-row gate/up pair without a fused norm at K = 8192 (norm launch first),
# q/k/v at K = 8192 as norm launch + grouped launch -- parity tests, the 70B / 8B layer chains and the
# 70B census; `bash r5_s8.sh ab`: the 70B decode on this tree and on the round-4 tree (_ab_r4) back to
# back on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
if [ "${1:-}" = ab ]; then
  rm -rf gpurun_out/r5m_*
  B70="--model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4"
  step r5m_bench70_new 400 python bench.py $B70
  (cd _ab_r4 && timeout -k 10 400 python bench.py $B70 > ../gpurun_out/r5m_bench70_r4.log 2>&1); rc=$?
  echo "== r5m_bench70_r4 rc=$rc"; tail -1 gpurun_out/r5m_bench70_r4.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
  step r5m_bench70_new2 400 python bench.py $B70
  echo done; exit 0
fi
rm -rf gpurun_out/r5l_*
step r5l_tests 500 python -u -m pytest tests/test_gpu_mlp_pair.py tests/test_gpu_layer_ops.py tests/test_gpu_prenorm.py tests/test_gpu_parity.py tests/test_gpu_mlp_chain.py -x -q --timeout 120 --timeout-method thread
step r5l_chain70 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5l_prof70 -o run --output-format csv -- python bench.py --model llama3-70b --chain-only
step r5l_chain8 240 python bench.py --chain-only
echo done
