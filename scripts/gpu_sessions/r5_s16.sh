#!/bin/bash
# round 5: greedy pick + feedback as one launch -- tests, A/B bench (kernel vs two-stage)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5g_*
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_glue.py > gpurun_out/r5g_tests.log 2>&1 || { tail -40 gpurun_out/r5g_tests.log; exit 1; }
tail -2 gpurun_out/r5g_tests.log
for i in 1 2; do
  for g in kernel two-stage; do
    timeout -k 10 300 python3 bench.py --greedy $g > gpurun_out/r5g_bench_${g}_$i.json 2> gpurun_out/r5g_bench_${g}_$i.log || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/r5g_bench_${g}_$i.json').read().strip().splitlines()[-1]); print('$g $i', d['value'], d['ms_per_step'])"
  done
done
echo done
