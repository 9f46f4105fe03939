#!/bin/bash
# round 3 measurement session: smoke, the bench lines (default = config #2 with the reference's
# fp32 compute_dtype -> exact codes; FP4 = config #3; 70B shapes on one GPU = config #5; bf16
# model), the 4096^2 GEMV kernel trace + FETCH / WRITE passes of the exact-code product kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3z_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r3z_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r3z_bench 600 python bench.py
step r3z_bench_fp4 300 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --steps 32 --warmup 4
step r3z_bench_70b 480 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline
step r3z_bench_bf16 300 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
step r3z_gemv_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3z_gemv_trace -- python3 bench.py --gemv-only
step r3z_gemv_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3z_gemv_fetch -- python3 bench.py --gemv-only
step r3z_gemv_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3z_gemv_write -- python3 bench.py --gemv-only
