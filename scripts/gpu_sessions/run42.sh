# add_rms_norm (residual add + post-attention norm in one launch): GPU parity, bench, TP path, batch 4
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E '^\{|passed|failed' "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || { grep -E "^E " "gpurun_out/$name.log" | head -5; exit $rc; }
}
step layer_ops_tests 300 python -u -m pytest tests/test_gpu_layer_ops.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_all 480 python bench.py
step bench_force_shard 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --force-shard --no-prefill --no-cpu --no-roofline
step bench_batch4 480 python bench.py --batch 4 --no-prefill --no-cpu --no-roofline
