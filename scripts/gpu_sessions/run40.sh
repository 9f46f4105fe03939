# silu_mul (LlamaMLP gate product in one launch): GPU parity, default bench line, ablation without it
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
step bench_no_mlp 300 python bench.py --no-prefill --no-cpu --no-roofline --layer-ops norm
