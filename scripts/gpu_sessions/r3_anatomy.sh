#!/bin/bash
# decode-step kernel census of the current default model layout (graph replay, 8B NF4+DQ)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3an; mkdir -p gpurun_out/r3an
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3an/trace -o run -- \
  python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline > gpurun_out/r3an/bench.log 2>&1
rc=$?; echo "== trace rc=$rc"; tail -2 gpurun_out/r3an/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python3 scripts/decode_anatomy.py gpurun_out/r3an/trace --steps 4 > gpurun_out/r3an/anatomy.txt 2>&1
rc=$?; head -60 gpurun_out/r3an/anatomy.txt
rm -rf gpurun_out/r3an/trace
exit $rc
