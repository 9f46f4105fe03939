#!/bin/bash
# latency-first decode attention (every global load issued up front, probabilities in their own
# buffer, 8-wide P V) and the two-stage greedy argmax: attention tests, the Llama greedy/graph
# tests, then same-box A/B bench lines (default, --torch-argmax) and a decode-step census
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3b_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r3b_attn_tests 300 python -u -m pytest tests/test_gpu_decode_attention.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step r3b_bench 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
step r3b_bench_torch_argmax 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes --torch-argmax
step r3b_bench2 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3b_an/trace -o run -- \
  python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r3b_an_bench.log 2>&1
rc=$?; echo "== trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/decode_anatomy.py gpurun_out/r3b_an/trace --steps 4 > gpurun_out/r3b_anatomy.txt 2>&1
rc=$?; cut -c1-160 gpurun_out/r3b_anatomy.txt | head -12
rm -rf gpurun_out/r3b_an
exit $rc
