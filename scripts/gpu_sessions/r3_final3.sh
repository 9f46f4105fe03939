#!/bin/bash
# round 3 closing session (after the attention / argmax changes): smoke, the whole GPU suite, the
# default bench line, FP4 / 70B-on-one-GPU / bf16 lines, 4096^2 GEMV kernel trace, decode census
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3f_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -2 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step r3f_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r3f_pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step r3f_attn_abl 240 python scripts/dev/attn_ablation.py
step r3f_bench 480 python bench.py
step r3f_bench_fp4 300 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --steps 32 --warmup 4
step r3f_bench_70b 480 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline
step r3f_bench_bf16 300 python bench.py --dtype bf16 --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4
step r3f_gemv_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f_gemv_trace -- python3 bench.py --gemv-only
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3f_an/trace -o run -- \
  python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r3f_an_bench.log 2>&1
rc=$?; echo "== trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/decode_anatomy.py gpurun_out/r3f_an/trace --steps 4 > gpurun_out/r3f_anatomy.txt 2>&1
rc=$?; cut -c1-160 gpurun_out/r3f_anatomy.txt | head -8
rm -rf gpurun_out/r3f_an
exit $rc
