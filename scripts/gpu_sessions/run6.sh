#!/bin/bash
# GPU parity + fused-group decode A/B + prefill crossover sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider
step bench_fused 300 python bench.py --steps 64 --warmup 8 --no-prefill --no-cpu --no-roofline
step bench_unfused 300 python bench.py --steps 64 --warmup 8 --no-prefill --no-cpu --no-roofline --no-fuse

