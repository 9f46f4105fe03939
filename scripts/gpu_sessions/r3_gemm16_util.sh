#!/bin/bash
# round 3: MFMA utilisation and clock of qz_gemm_16bit vs hipBLASLt at config #4 (4096^2, T = 16384)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3u_*
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3u_trace -o run -- python3 scripts/prof_prefill.py 20 gemm16,dequant > gpurun_out/r3u_trace.log 2>&1 || { tail -20 gpurun_out/r3u_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r3u_pmc -o run -- python3 scripts/prof_prefill.py 20 gemm16,dequant > gpurun_out/r3u_pmc.log 2>&1 || { tail -20 gpurun_out/r3u_pmc.log; exit 1; }
T=$(find gpurun_out/r3u_trace -name "*kernel_trace.csv" | head -1); P=$(find gpurun_out/r3u_pmc -name "*counter_collection.csv" | head -1)
python3 scripts/mfma_util.py "$P" "$T" | tee gpurun_out/r3u_util.txt
