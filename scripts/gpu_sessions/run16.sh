set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --quant fp4 --no-dq --no-prefill --no-cpu --no-roofline > gpurun_out/bench_fp4.log 2>&1; rc=$?; tail -1 gpurun_out/bench_fp4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python bench.py --model llama3-70b --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline > gpurun_out/bench_70b.log 2>&1; rc=$?; tail -2 gpurun_out/bench_70b.log; exit $rc
