#!/bin/bash
# round 5, closing: the Linear4bit chain on one rank's rows at N = 1/2/4/8 on the final tree, 70B and 8B
# (the DESIGN 6 budgets)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5v_*
for m in llama3-70b llama3-8b; do
  for n in 1 2 4 8; do
    timeout -k 10 240 python3 bench.py --model $m --chain-only --chain-shards $n > gpurun_out/r5v_${m}_n$n.log 2>&1 || exit $?
    grep -o '"us_per_layer": [0-9.]*' gpurun_out/r5v_${m}_n$n.log | sed "s/^/$m N=$n /"
  done
done
echo done
