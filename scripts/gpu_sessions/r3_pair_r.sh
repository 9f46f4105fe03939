#!/bin/bash
# gate/up pair launch rows per wave (QZ_PAIR_R = 2 / 3 / 4): bit-identity at R = 3 and 2, launch
# times, same-box bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3g_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -2 | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
QZ_PAIR_R=3 step r3g_pair_tests_r3 300 python -u -m pytest tests/test_gpu_mlp_pair.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
QZ_PAIR_R=2 step r3g_pair_tests_r2 300 python -u -m pytest tests/test_gpu_mlp_pair.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
QZ_PAIR_R=2 step r3g_times_r2 200 python scripts/dev/pair_times.py
QZ_PAIR_R=3 step r3g_times_r3 200 python scripts/dev/pair_times.py
QZ_PAIR_R=4 step r3g_times_r4 200 python scripts/dev/pair_times.py
QZ_PAIR_R=3 step r3g_bench_r3 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
QZ_PAIR_R=4 step r3g_bench_r4 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
QZ_PAIR_R=2 step r3g_bench_r2 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
