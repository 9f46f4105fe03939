# SQ counters: LDS byte-table GEMV vs v_perm GEMV (microbench, 28672x4096 and 4096^2)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for shp in "28672 4096" "4096 4096"; do
  set -- $shp
  for c in 1 2; do
    eval CC=\$C$c
    rm -rf gpurun_out/tpmc${c}_$1x$2
    timeout -k 10 300 rocprofv3 --pmc $CC --output-format csv -d gpurun_out/tpmc${c}_$1x$2 -- scripts/microbench/gemv_micro $1 $2 1 tab > gpurun_out/tpmc${c}_$1x$2.log 2>&1; rc=$?
    echo "== pmc$c $1x$2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tpmc${c}_$1x$2.log; exit $rc; }
  done
done
find gpurun_out/tpmc* -name "*counter_collection.csv" | head
