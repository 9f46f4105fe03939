#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_prenorm.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3p_tests.log 2>&1 || { tail -40 gpurun_out/r3p_tests.log; exit 1; }
tail -1 gpurun_out/r3p_tests.log
timeout -k 10 480 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline > gpurun_out/r3p_70b.log 2>&1 || { tail -5 gpurun_out/r3p_70b.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r3p_70b.log | head -1
