set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/microbench/gemv_micro 4096 4096 > gpurun_out/micro.log 2>&1; echo "micro rc=$?"; cat gpurun_out/micro.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_micro -- ./scripts/microbench/gemv_micro 4096 4096 > gpurun_out/prof_micro.log 2>&1; echo "prof rc=$?"
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -k "golden or graph or tiny" -p no:cacheprovider > gpurun_out/pytest_sel.log 2>&1; echo "pytest rc=$?"; tail -15 gpurun_out/pytest_sel.log
timeout -k 10 300 python bench.py --steps 32 --warmup 4 --no-cpu > gpurun_out/bench3.log 2>&1; echo "bench rc=$?"; tail -4 gpurun_out/bench3.log
