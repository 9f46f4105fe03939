#!/bin/bash
# round 3: RMSNorm absorbed into the grouped decode GEMV: parity tests, then bench with / without
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r3p_*
timeout -k 10 400 python -u -m pytest tests/test_gpu_prenorm.py tests/test_gpu_layer_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3p_tests.log 2>&1 || { tail -40 gpurun_out/r3p_tests.log; exit 1; }
tail -2 gpurun_out/r3p_tests.log
timeout -k 10 400 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r3p_bench.log 2>&1 || { tail -20 gpurun_out/r3p_bench.log; exit 1; }
timeout -k 10 400 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes --no-prenorm > gpurun_out/r3p_bench_noprenorm.log 2>&1 || { tail -20 gpurun_out/r3p_bench_noprenorm.log; exit 1; }
grep -h -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r3p_bench.log gpurun_out/r3p_bench_noprenorm.log
