set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --pmc $C1 --output-format csv -d gpurun_out/gpmc1 -- python3 scripts/prof_gemm.py 16384 4096 4096 > gpurun_out/gpmc1.log 2>&1; echo "pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/gpmc2 -- python3 scripts/prof_gemm.py 16384 4096 4096 > gpurun_out/gpmc2.log 2>&1; echo "pmc2 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gtrace -- python3 scripts/prof_gemm.py 16384 4096 4096 > gpurun_out/gtrace.log 2>&1; echo "trace rc=$?"
timeout -k 10 200 python bench.py --gemv-only > gpurun_out/gemv_only.log 2>&1; echo "gemv rc=$?"; tail -1 gpurun_out/gemv_only.log
