#!/bin/bash
# round 6: same-box A/B of the Llama-3-70B one-GPU decode bench line, this tree (A) against the round-5 tree (B, a git worktree
# of 22fd24c built in-tree under _ab_r5): A B A B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ARGS="--model llama3-70b --no-prefill --no-cpu --no-roofline --no-extra-codes --no-extra-weak"
for i in 1 2; do
  timeout -k 10 500 python3 -u bench.py $ARGS > gpurun_out/r6_ab70_A$i.json 2> gpurun_out/r6_ab70_A$i.err || { tail -3 gpurun_out/r6_ab70_A$i.err; exit 1; }
  (cd _ab_r5 && timeout -k 10 500 python3 -u bench.py $ARGS > ../gpurun_out/r6_ab70_B$i.json 2> ../gpurun_out/r6_ab70_B$i.err) || { tail -3 gpurun_out/r6_ab70_B$i.err; exit 1; }
done
for f in A1 B1 A2 B2; do python3 -c "
import json; l=json.loads(open('gpurun_out/r6_ab70_$f.json').read().strip().splitlines()[-1]); print('$f', l['value'], l['ms_per_step'])"; done
