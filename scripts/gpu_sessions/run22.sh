set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -q -x -p no:cacheprovider -k "multi_token or gemm" > gpurun_out/pytest_mt.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_mt.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/mttrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mttrace -- python3 scripts/prof_gemm.py 8 4096 4096 nf4 20 > gpurun_out/mttrace.log 2>&1; echo "trace rc=$?"
