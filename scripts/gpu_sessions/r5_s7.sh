#!/bin/bash
# round 5, session 7: K = 8192 (Llama-3-70B) launch geometry sweep (gemv_micro geom8k) and the q/k/v /
# o_proj / gate-up launch forms at 70B shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5j_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r5j_geom_o 120 scripts/microbench/gemv_micro 8192 8192 7 geom8k
step r5j_geom_qkv 120 scripts/microbench/gemv_micro 10240 8192 7 geom8k
step r5j_geom_gu 300 scripts/microbench/gemv_micro 57344 8192 5 geom8k
step r5j_qkv70 240 python scripts/dev/qkv70_times.py
step r5j_split 240 python scripts/dev/pair_split_times.py
echo done
