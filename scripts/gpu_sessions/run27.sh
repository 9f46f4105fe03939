# SQ counters for the byte-table GEMV variants (microbench mode ${MODE:-tabfs})
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for shp in ${SHAPES:-"4096 4096" "28672 4096"}; do
  set -- $shp
  for c in 1 2; do
    eval CC=\$C$c
    rm -rf gpurun_out/tpmc${c}_$1x$2
    timeout -k 10 300 rocprofv3 --pmc $CC --output-format csv -d gpurun_out/tpmc${c}_$1x$2 -- scripts/microbench/gemv_micro $1 $2 1 ${MODE:-tabfs} > gpurun_out/tpmc${c}_$1x$2.log 2>&1; rc=$?
    echo "== pmc$c $1x$2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/tpmc${c}_$1x$2.log; exit $rc; }
  done
done
