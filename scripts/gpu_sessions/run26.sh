# GEMV microbench runs: MODE selects the variant set, SHAPES lists M_K pairs
set -u
cd $GRAFT_REPO_ROOT/scripts/microbench
for sh in ${SHAPES:-4096_4096 28672_4096 8192_28672}; do
  s=${sh//_/ }
  timeout -k 10 120 ./gemv_micro $s 7 ${MODE:-tabab} > ../../gpurun_out/mb_${MODE:-tabab}_${sh}.log 2>&1; rc=$?
  echo "== $s rc=$rc"; grep -v "^floor T=256 L=1" ../../gpurun_out/mb_${MODE:-tabab}_${sh}.log
  [ $rc -eq 0 ] || exit $rc
done
