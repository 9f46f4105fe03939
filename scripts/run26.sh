# ablations of the LDS byte-table GEMV decode
set -u
cd $GRAFT_REPO_ROOT/scripts/microbench
for s in ${SHAPES:-"4096 4096" "28672 4096" "8192 28672"}; do
  timeout -k 10 120 ./gemv_micro $s 7 ${MODE:-tabab} > ../../gpurun_out/tabab_${s// /x}.log 2>&1; rc=$?
  echo "== $s rc=$rc"; grep -v "^floor T=256 L=1" ../../gpurun_out/tabab_${s// /x}.log
  [ $rc -eq 0 ] || exit $rc
done
