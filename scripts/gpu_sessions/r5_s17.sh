#!/bin/bash
# round 5: the fp16 lm_head on qz_gemv_dense -- tests, A/B bench (dense vs hipBLASLt), 8B and 70B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5h_*
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_glue.py > gpurun_out/r5h_tests.log 2>&1 || { tail -40 gpurun_out/r5h_tests.log; exit 1; }
tail -2 gpurun_out/r5h_tests.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['value'], d['ms_per_step'], d['config'].get('lm_head'))"; }
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-prefill --no-cpu > gpurun_out/r5h_dense_$i.json 2> gpurun_out/r5h_dense_$i.log || exit $?
  show gpurun_out/r5h_dense_$i.json "8B dense $i"
  timeout -k 10 300 python3 bench.py --no-prefill --no-cpu --lm-head-library > gpurun_out/r5h_lib_$i.json 2> gpurun_out/r5h_lib_$i.log || exit $?
  show gpurun_out/r5h_lib_$i.json "8B library $i"
done
B70="--model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4"
timeout -k 10 400 python3 bench.py $B70 > gpurun_out/r5h_70_dense.json 2> gpurun_out/r5h_70_dense.log || exit $?
show gpurun_out/r5h_70_dense.json "70B dense"
timeout -k 10 400 python3 bench.py $B70 --lm-head-library > gpurun_out/r5h_70_lib.json 2> gpurun_out/r5h_70_lib.log || exit $?
show gpurun_out/r5h_70_lib.json "70B library"
echo done
