set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/ptrace2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ptrace2 -- python3 scripts/prof_prefill.py > gpurun_out/ptrace2.log 2>&1; echo "trace rc=$?"
