#!/bin/bash
# round 2, session 1: exact-code GEMV, activation range, config #4 full size, oracle checkpoint; bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_exact.py tests/test_gpu_config4.py tests/test_checkpoint.py \
  "tests/test_gpu_parity.py::test_linear4bit_bf16_fp32_activations_and_compute_dtype" \
  > gpurun_out/r2_new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -15 gpurun_out/r2_new_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 32 --warmup 4 > gpurun_out/r2_bench1.json 2> gpurun_out/r2_bench1.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r2_bench1.err; cat gpurun_out/r2_bench1.json
exit $rc
