set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider -k "gemm or linear4bit or llama" > gpurun_out/pytest_gemm.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --prefill-sweep > gpurun_out/prefill_sweep2.log 2>&1; rc=$?; tail -1 gpurun_out/prefill_sweep2.log; exit $rc
