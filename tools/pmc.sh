#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, --kernel-trace only; never with sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="${BENCH_ARGS:---no-cpu --no-train --no-pmc --steps 3 --warmup 1}"
if [ "${LIST:-0}" = "1" ]; then
  timeout -k 5 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
fi
i=0
IFS=';'
for grp in ${PASSES:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR}; do
  i=$((i+1))
  unset IFS
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- python bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  IFS=';'
  [ $rc -eq 0 ] || { echo "pmc pass $i ($grp) failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; }
  echo "pass $i ok: $grp"
done
