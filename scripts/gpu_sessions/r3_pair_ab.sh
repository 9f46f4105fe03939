#!/bin/bash
# one box: the gate/up + SiLU pair launch on / off, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3pa
for i in 1 2; do
  for v in pair nopair; do
    extra=""; [ $v = nopair ] && extra="--no-mlp-pair"
    timeout -k 10 300 python bench.py --no-prefill --no-cpu --no-roofline --no-extra-codes $extra > gpurun_out/r3pa/$v$i.log 2>&1 || exit 1
    echo "$v$i $(grep -o '"value": [0-9.]*' gpurun_out/r3pa/$v$i.log | head -1)"
  done
done
