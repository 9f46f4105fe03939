#!/bin/bash
# round 2 profiles: GEMV roofline kernel trace + FETCH/WRITE PMC passes (exact-code
# product kernel and the fp16-code one), prefill MFMA utilisation (8-phase kernel vs
# dequant+hipBLASLt), the default N>1 bench layout at world size 1 (RCCL, graph capture)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r2p_*
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step r2p_gemv_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2p_gemv_trace -- python3 bench.py --gemv-only
step r2p_gemv_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2p_gemv_fetch -- python3 bench.py --gemv-only
step r2p_gemv_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2p_gemv_write -- python3 bench.py --gemv-only
step r2p_prefill_pmc 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r2p_prefill_pmc -- python3 scripts/prof_prefill.py
step r2p_prefill_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2p_prefill_trace -- python3 scripts/prof_prefill.py
step r2p_tp1_gather 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --force-shard --steps 32 --warmup 4 --no-prefill --no-cpu --no-roofline
step r2p_tp1_weak 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 1 --force-shard --weak --steps 32 --warmup 4 --no-prefill --no-cpu --no-roofline
