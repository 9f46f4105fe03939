#!/bin/bash
# round 6: the GPU suite, smoke() and a default bench line on the current tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_smoke.log 2>&1 || { tail -5 gpurun_out/r6_smoke.log; exit 1; }
tail -1 gpurun_out/r6_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err || { tail -5 gpurun_out/r6_bench.err; exit 1; }
python3 -c "
import json; l=json.loads(open('gpurun_out/r6_bench.json').read().strip().splitlines()[-1])
print(l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline'].get('dominant_decode_kernel',{}).get('frac'))"
