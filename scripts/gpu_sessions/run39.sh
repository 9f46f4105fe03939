# configs #3 (FP4, no double quant) and #5 (70B NF4+DQ, one GPU) with the layer ops
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || { tail -5 "gpurun_out/$name.log"; exit $rc; }
}
step bench_cfg3_fp4 480 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu
step bench_cfg5_70b 900 python bench.py --model llama3-70b --no-prefill --no-cpu --steps 32 --warmup 4
