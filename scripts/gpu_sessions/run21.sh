set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/mttrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mttrace -- python3 scripts/prof_gemm.py 8 4096 4096 nf4 20 > gpurun_out/mttrace.log 2>&1; echo "trace rc=$?"
