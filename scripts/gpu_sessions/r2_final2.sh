#!/bin/bash
# round 2 closing run: smoke, the whole GPU suite, the bench lines (default = config #2, FP4 =
# config #3, 70B shapes on one GPU = config #5, bf16 model), the GEMV kernel trace + FETCH /
# WRITE PMC passes of the product kernel, the tp1 row-split layout
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r2z_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r2z_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r2z_pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r2z_bench 480 python bench.py
step r2z_bench_fp4 300 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --steps 32 --warmup 4
step r2z_bench_70b 480 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline
step r2z_bench_bf16 300 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
step r2z_gemv_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2z_gemv_trace -- python3 bench.py --gemv-only
step r2z_gemv_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2z_gemv_fetch -- python3 bench.py --gemv-only
step r2z_gemv_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2z_gemv_write -- python3 bench.py --gemv-only
step r2z_tp1_gather 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-shard --steps 32 --warmup 4 --no-prefill --no-cpu --no-extra-weak
