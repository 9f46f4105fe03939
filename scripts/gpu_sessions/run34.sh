# layer ops (one-launch RMSNorm + q/k rotary): GPU parity, then the default bench line
# with and without them
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step layer_ops_tests 300 python -u -m pytest tests/test_gpu_layer_ops.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_layer_ops 480 python bench.py --no-prefill
step bench_no_layer_ops 480 python bench.py --no-prefill --no-cpu --no-roofline --no-layer-ops
