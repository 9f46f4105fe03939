#!/bin/bash
# round 5, session 11: the 8192 x 8192 launch at R = 2 with whole rows (70B o_proj) -- parity tests
# touching it, the down_proj geometry sweep at K = 28672, and the 70B decode A/B against the round-4
# tree (_ab_r4) on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5q_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r5q_tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exact.py tests/test_gpu_residual.py tests/test_gpu_xgmi_rowsplit.py -x -q --timeout 120 --timeout-method thread
step r5q_geom_down 200 scripts/microbench/gemv_micro 8192 28672 5 geom
B70="--model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4"
step r5q_bench70_new 400 python bench.py $B70
(cd _ab_r4 && timeout -k 10 400 python bench.py $B70 > ../gpurun_out/r5q_bench70_r4.log 2>&1); rc=$?
echo "== r5q_bench70_r4 rc=$rc"; tail -1 gpurun_out/r5q_bench70_r4.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
step r5q_bench70_new2 400 python bench.py $B70
echo done
