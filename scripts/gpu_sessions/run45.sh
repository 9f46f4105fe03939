# after templating the multi-token kernel on waves per workgroup (product still W = 8): multi-token
# parity tests, smoke
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "multi_token or grouped or tiny_llama" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mt_tests.log 2>&1 || { tail -20 gpurun_out/mt_tests.log; exit 1; }
tail -1 gpurun_out/mt_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
