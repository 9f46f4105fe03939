#!/bin/bash
# q/k/v grouped launch with the fused pre-norm at 1 / 2 / 4 rows per wave (QZ_GROUPED_NORM_R)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3i_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -3 | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
QZ_GROUPED_NORM_R=4 step r3i_prenorm_tests_r4 300 python -u -m pytest tests/test_gpu_prenorm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
QZ_GROUPED_NORM_R=2 step r3i_times_r2 200 python scripts/dev/prenorm_times.py
QZ_GROUPED_NORM_R=4 step r3i_times_r4 200 python scripts/dev/prenorm_times.py
QZ_GROUPED_NORM_R=1 step r3i_times_r1 200 python scripts/dev/prenorm_times.py
QZ_GROUPED_NORM_R=4 step r3i_bench_r4 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
step r3i_bench_def 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
