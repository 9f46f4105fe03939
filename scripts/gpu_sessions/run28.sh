# Round-1 evidence refresh: rocprofv3 GEMV passes + decode trace, default bench, configs #3 and #5
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DECODE_CMD="python3 bench.py --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline" bash scripts/gpu_profile.sh || exit $?
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step bench_full 420 python bench.py
step bench_cfg3 300 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --no-roofline
step bench_cfg5 420 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline
