#!/bin/bash
# decode-step census of the fully fused step (attention, residual epilogues, gate/up pair)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
rm -rf gpurun_out/r3an2; mkdir -p gpurun_out/r3an2
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3an2/trace -o run -- \
  python3 bench.py --steps 8 --warmup 4 --no-prefill --no-cpu --no-roofline --no-extra-codes > gpurun_out/r3an2/bench.log 2>&1
rc=$?; echo "== trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/decode_anatomy.py gpurun_out/r3an2/trace --steps 4 > gpurun_out/r3an2/anatomy.txt 2>&1
rc=$?; cut -c1-180 gpurun_out/r3an2/anatomy.txt | head -30
rm -rf gpurun_out/r3an2/trace
exit $rc
