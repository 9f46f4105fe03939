#!/bin/bash
# round 5, closing (after the glue, the dense lm_head and the greedy launches): whole GPU suite +
# smoke, then the bench lines (8B default, FP4, bf16); `r5_final3.sh 70b`: the 70B A/B against the
# round-4 tree on one box, and the 70B census
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
}
if [ "${1:-}" = 70b ]; then
  rm -rf gpurun_out/r5k_*
  B70="--model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4"
  step r5k_bench70_new 400 python bench.py $B70
  (cd _ab_r4 && timeout -k 10 400 python bench.py $B70 > ../gpurun_out/r5k_bench70_r4.log 2>&1); rc=$?
  echo "== r5k_bench70_r4 rc=$rc"; tail -1 gpurun_out/r5k_bench70_r4.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
  step r5k_bench70_new2 400 python bench.py $B70
  step r5k_an70 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5k_an70/trace -- python3 bench.py --model llama3-70b --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes
  python3 scripts/decode_anatomy.py gpurun_out/r5k_an70/trace --steps 4 > gpurun_out/r5k_anatomy70.txt 2>&1 || exit $?
  rm -rf gpurun_out/r5k_an70/trace
  head -12 gpurun_out/r5k_anatomy70.txt | cut -c1-150
  echo done; exit 0
fi
bash scripts/gpu_sessions/r5_final_tests.sh || exit $?
rm -rf gpurun_out/r5j_*
step r5j_bench 600 python bench.py
step r5j_bench_fp4 400 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --no-roofline
step r5j_bench_bf16 400 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline
echo done
