#!/bin/bash
# round 4, session 3: GEMV timeline stamps (product vs early second step vs SGPR table); the
# fused decoder layer on row shards (GPU tests at world 2, sharded pair at R = 1, residual
# fallback, full-cache attention); world-1 force-shard bench vs the single-GPU line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r4c_stamps 200 ./scripts/microbench/gemv_micro 4096 4096 9 stamps
for s in "4096 4096" "14336 4096" "28672 4096" "6144 4096"; do
  set -- $s
  step r4c_mf_$1x$2 200 ./scripts/microbench/gemv_micro $1 $2 7 mf
done
step r4c_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_mlp_pair.py tests/test_gpu_residual.py tests/test_gpu_decode_attention.py tests/test_gpu_prenorm.py \
  tests/test_gpu_xgmi_rowsplit.py tests/test_gpu_xgmi_exchange.py
step r4c_bench1 400 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes --steps 64
step r4c_bench_fs1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --force-shard --no-prefill --no-cpu --no-roofline --no-extra-weak --steps 64
echo done
