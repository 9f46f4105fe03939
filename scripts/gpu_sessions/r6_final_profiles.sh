#!/bin/bash
# round 6, closing: rocprofv3 on the bench line's cited launches as the final tree runs them (the 4096^2
# roofline GEMV, the dominant gate/up pair: kernel trace + FETCH / WRITE passes), the decode-token census,
# and the attention launch at the head counts of the head-sharded row split
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r6y_*
pmc() {  # name cmd... (one rocprofv3 pass, killed hard at 150 s)
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pmc r6y_gemv_trace --kernel-trace --stats --output-format csv -d gpurun_out/r6y_gemv_trace -- python3 bench.py --gemv-only
pmc r6y_gemv_fetch --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6y_gemv_fetch -- python3 bench.py --gemv-only
pmc r6y_gemv_write --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6y_gemv_write -- python3 bench.py --gemv-only
pmc r6y_dom_trace --kernel-trace --stats --output-format csv -d gpurun_out/r6y_dom_trace -- python3 bench.py --dominant-only
for d in r6y_gemv_fetch r6y_gemv_write r6y_gemv_trace; do
  python3 scripts/rocprof_summary.py gpurun_out/$d --match k_gemv_4bit --json gpurun_out/$d.json > gpurun_out/$d.summary.txt 2>&1 || exit $?
done
python3 scripts/rocprof_summary.py gpurun_out/r6y_dom_trace --match pair --json gpurun_out/r6y_dom_trace.json > gpurun_out/r6y_dom_trace.summary.txt 2>&1 || exit $?
head -4 gpurun_out/r6y_gemv_fetch.summary.txt gpurun_out/r6y_gemv_trace.summary.txt gpurun_out/r6y_dom_trace.summary.txt | cut -c1-220
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6y_an8/trace -- python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r6y_an8.log 2>&1 || exit $?
python3 scripts/decode_anatomy.py gpurun_out/r6y_an8/trace --steps 4 > gpurun_out/r6y_anatomy8.txt 2>&1 || exit $?
head -8 gpurun_out/r6y_anatomy8.txt | cut -c1-200
timeout -k 10 200 python3 -u scripts/attn_heads_times.py > gpurun_out/r6y_attn_heads.txt 2>&1 || exit $?
grep -v '^{' gpurun_out/r6y_attn_heads.txt
echo done
