#!/bin/bash
# rocprofv3 PMC passes over tools/flow_time.py (one counter group per pass, --kernel-trace only, never
# with sys/runtime trace). VAR="ENF_X=1 ..." selects a diagnostics-library variant; PRODUCT=1 the
# shipping library. Writes gpurun_out/pmc_<TAG>/p<i>/.
set -u
OUT=gpurun_out/pmc_${TAG:-flow}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="--steps 3 ${FLOW_ARGS:-} ${PRODUCT:+--product}"
if [ "${LIST:-0}" = "1" ]; then
  timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
fi
i=0
IFS=';'
for grp in ${PASSES:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE;SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC}; do
  i=$((i+1))
  unset IFS
  env ${VAR:-ENF_NONE=0} timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- python tools/flow_time.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  IFS=';'
  [ $rc -eq 0 ] || { echo "pmc pass $i ($grp) failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; }
  echo "pass $i ok: $grp"
done
