#!/bin/bash
# round 5, closing: where a decode token goes on the final tree (8B, and 70B on one GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r5w_*
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5w_an8/trace -- python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r5w_an8.log 2>&1 || exit $?
python3 scripts/decode_anatomy.py gpurun_out/r5w_an8/trace --steps 4 > gpurun_out/r5w_anatomy8.txt 2>&1 || exit $?
head -14 gpurun_out/r5w_anatomy8.txt | cut -c1-200
timeout -s KILL 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5w_an70/trace -- python3 bench.py --model llama3-70b --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r5w_an70.log 2>&1 || exit $?
python3 scripts/decode_anatomy.py gpurun_out/r5w_an70/trace --steps 4 > gpurun_out/r5w_anatomy70.txt 2>&1 || exit $?
head -14 gpurun_out/r5w_anatomy70.txt | cut -c1-200
timeout -k 10 200 scripts/microbench/gemv_micro 4096 14336 5 geom > gpurun_out/r5w_geom_down8b.log 2>&1 || exit $?
grep median gpurun_out/r5w_geom_down8b.log | cut -c1-120
echo done
