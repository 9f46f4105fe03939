# LDS byte-table GEMV decode (kModeTab) vs v_perm decode, microbench shapes
set -u
cd $GRAFT_REPO_ROOT/scripts/microbench
for s in "4096 4096" "6144 4096" "28672 4096" "4096 14336" "8192 28672"; do
  timeout -k 10 120 ./gemv_micro $s 7 tab > ../../gpurun_out/tab_${s// /x}.log 2>&1; rc=$?
  echo "== $s rc=$rc"; cat ../../gpurun_out/tab_${s// /x}.log
  [ $rc -eq 0 ] || exit $rc
done
