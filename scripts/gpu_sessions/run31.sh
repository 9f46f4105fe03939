# config #4 prefill after the 256x256 tile kernel: MFMA-utilisation PMC pass + kernel trace
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/ppmc gpurun_out/ptrace
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ppmc -- python3 scripts/prof_prefill.py > gpurun_out/ppmc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ptrace -- python3 scripts/prof_prefill.py > gpurun_out/ptrace.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --prefill-only > gpurun_out/prefill_only.log 2>&1 || exit $?
tail -2 gpurun_out/prefill_only.log
