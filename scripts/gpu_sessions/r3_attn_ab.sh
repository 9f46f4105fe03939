#!/bin/bash
# fused decode attention on/off on one box, then the decode-step census with it on
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3ab; mkdir -p gpurun_out/r3ab
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/r3ab/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/r3ab/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step bench_attn 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
step bench_noattn 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes --no-attention
step bench_attn2 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
step trace 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3ab/trace -o run -- python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes
python3 scripts/decode_anatomy.py gpurun_out/r3ab/trace --steps 4 > gpurun_out/r3ab/anatomy.txt 2>&1
rc=$?; head -40 gpurun_out/r3ab/anatomy.txt | cut -c1-200
rm -rf gpurun_out/r3ab/trace
exit $rc
