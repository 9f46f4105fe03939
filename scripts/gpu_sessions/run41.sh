# round-1 final refresh with the layer ops: smoke, full GPU suite, default bench line,
# rocprofv3 kernel-trace of the GEMV roofline command and of the decode step
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_final 480 python bench.py
rm -rf gpurun_out/gemv_trace gpurun_out/decode_trace
step gemv_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gemv_trace -- python3 bench.py --gemv-only
step decode_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/decode_trace -- python3 bench.py --steps 16 --warmup 4 --no-prefill --no-cpu --no-roofline
