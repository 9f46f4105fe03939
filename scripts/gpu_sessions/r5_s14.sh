#!/bin/bash
# round 5: decode-step glue (causal mask + rotary tables, one launch each) -- tests, A/B bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5x_*
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_glue.py > gpurun_out/r5x_tests.log 2>&1 || { tail -40 gpurun_out/r5x_tests.log; exit 1; }
tail -2 gpurun_out/r5x_tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py > gpurun_out/r5x_bench_glue$i.json 2> gpurun_out/r5x_bench_glue$i.log || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/r5x_bench_glue$i.json | sed "s/^/glue $i /"
  timeout -k 10 300 python3 bench.py --no-glue > gpurun_out/r5x_bench_noglue$i.json 2> gpurun_out/r5x_bench_noglue$i.log || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/r5x_bench_noglue$i.json | sed "s/^/no-glue $i /"
done
echo done
