# final tree check: smoke, full GPU suite, default bench line
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_final 480 python bench.py
