#!/bin/bash
# round 5, session 9: (a) the 70B decode census (rocprofv3 kernel trace of bench.py's graph decode);
# (b) the 70B layer chain on one rank's rows at N = 1/2/4/8 with this round's forms (the DESIGN 6
# budget); (c) counters on the two 4096-row launches of the 8B decode (q/k/v + fused norm, o_proj +
# residual): SQ, FETCH, WRITE passes and a kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5o_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
pmc() {  # name cmd... (one PMC pass, killed hard at 120 s)
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
step r5o_pair70 300 python3 scripts/dev/pair_split_times.py
step r5o_census70 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5o_census70 -o run --output-format csv -- python3 bench.py --model llama3-70b --no-prefill --no-cpu --no-roofline --steps 16 --warmup 4
for n in 1 2 4 8; do
  step r5o_chain70_n$n 240 python3 bench.py --model llama3-70b --chain-only --chain-shards $n
done
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY"
pmc r5o_sq --pmc $SQ --output-format csv -d gpurun_out/r5o_sq -- python3 scripts/dev/qkv_o_launches.py 200
pmc r5o_fetch --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5o_fetch -- python3 scripts/dev/qkv_o_launches.py 200
pmc r5o_write --pmc WRITE_SIZE --output-format csv -d gpurun_out/r5o_write -- python3 scripts/dev/qkv_o_launches.py 200
pmc r5o_trace --kernel-trace --stats --output-format csv -d gpurun_out/r5o_trace -- python3 scripts/dev/qkv_o_launches.py 200
for d in r5o_sq r5o_fetch r5o_write r5o_trace; do
  python3 scripts/rocprof_summary.py gpurun_out/$d --match gemv --json gpurun_out/$d.json > gpurun_out/$d.summary.txt 2>&1 || exit $?
done
echo done
