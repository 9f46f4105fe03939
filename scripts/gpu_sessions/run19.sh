set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/ptrace3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ptrace3 -- python3 scripts/prof_prefill.py > gpurun_out/ptrace3.log 2>&1; echo "trace rc=$?"
