set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -m pytest tests/test_gpu_rounding.py -q -s -p no:cacheprovider > gpurun_out/pytest_round.log 2>&1; echo "rc=$?"; tail -15 gpurun_out/pytest_round.log
