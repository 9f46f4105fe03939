#!/bin/bash
# gate/up pair launch at 6 and 8 rows per wave (QZ_PAIR_R): bit-identity, launch times, bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3h_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -2 | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
QZ_PAIR_R=8 step r3h_pair_tests_r8 300 python -u -m pytest tests/test_gpu_mlp_pair.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
QZ_PAIR_R=6 step r3h_pair_tests_r6 300 python -u -m pytest tests/test_gpu_mlp_pair.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
QZ_PAIR_R=4 step r3h_times_r4 200 python scripts/dev/pair_times.py
QZ_PAIR_R=6 step r3h_times_r6 200 python scripts/dev/pair_times.py
QZ_PAIR_R=8 step r3h_times_r8 200 python scripts/dev/pair_times.py
QZ_PAIR_R=8 step r3h_bench_r8 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
QZ_PAIR_R=4 step r3h_bench_r4 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
QZ_PAIR_R=6 step r3h_bench_r6 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
