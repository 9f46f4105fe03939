#!/bin/bash
# round 5: the norm launch with a decode row's output spread over several workgroups -- 70B decode
# on this tree and on HEAD before the change (_ab_head worktree) back to back on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5s_*
B70="--model llama3-70b --no-prefill --no-cpu --no-roofline --steps 32 --warmup 4"
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['value'], d['ms_per_step'])"; }
for i in 1 2; do
  timeout -k 10 400 python3 bench.py $B70 > gpurun_out/r5s_new_$i.log 2>&1 || exit $?
  show gpurun_out/r5s_new_$i.log "sliced norm $i"
  (cd _ab_head && timeout -k 10 400 python3 bench.py $B70 > ../gpurun_out/r5s_old_$i.log 2>&1) || exit $?
  show gpurun_out/r5s_old_$i.log "one-workgroup norm $i"
done
echo done
