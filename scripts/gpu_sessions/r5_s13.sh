#!/bin/bash
# round 5: fused norm back for row-shard q/k/v at K-split geometries -- tests + shard chains
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5w_*
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_prenorm.py tests/test_gpu_mlp_pair.py > gpurun_out/r5w_tests.log 2>&1 || { tail -30 gpurun_out/r5w_tests.log; exit 1; }
tail -2 gpurun_out/r5w_tests.log
for mn in "llama3-8b 4" "llama3-8b 8" "llama3-70b 8" "llama3-70b 2" "llama3-8b 1"; do
  set -- $mn
  timeout -k 10 240 python3 bench.py --model $1 --chain-only --chain-shards $2 > gpurun_out/r5w_$1_n$2.log 2>&1 || exit $?
  echo "$1 N=$2 $(grep -o '"gate_up_form": \[[^]]*\]' gpurun_out/r5w_$1_n$2.log) $(grep -o '"us_per_layer": [0-9.]*' gpurun_out/r5w_$1_n$2.log)"
done
echo done
