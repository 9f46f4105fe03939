set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -q -x -p no:cacheprovider -k "multi_token" > gpurun_out/pytest_mt.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_mt.log; [ $rc -eq 0 ] || exit $rc
for T in 2 16; do
rm -rf gpurun_out/mt$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mt$T -- python3 scripts/prof_gemm.py $T 4096 4096 nf4 20 > gpurun_out/mt$T.log 2>&1; echo "trace $T rc=$?"
done
