#!/bin/bash
# round 5, session 5: the 70B decode A/B on one box (pair at K = 8192 vs the round-4 grouped form)
# and the kernel census of the 70B layer chain in both forms
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5e_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step r5e_prof70 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e_prof70 -o run -- python bench.py --model llama3-70b --chain-only
export QZ_PAIR_WK1=0
step r5e_prof70_old 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e_prof70_old -o run -- python bench.py --model llama3-70b --chain-only
unset QZ_PAIR_WK1
step r5e_bench70 420 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
export QZ_PAIR_WK1=0
step r5e_bench70_old 420 python bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
echo done
