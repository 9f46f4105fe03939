#!/bin/bash
# round 3: compute_dtype / exact-code tests, bench line (in-kernel stamps, both code tables),
# rocprofv3 kernel trace + FETCH/WRITE passes of the grouped gate/up launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3c_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r3c_tests 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_edges.py tests/test_checkpoint.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r3c_bench 600 python bench.py
step r3c_dom_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c_dom_trace -- python3 bench.py --dominant-only
step r3c_dom_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3c_dom_fetch -- python3 bench.py --dominant-only
step r3c_dom_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3c_dom_write -- python3 bench.py --dominant-only
