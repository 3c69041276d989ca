#!/bin/bash
# Effective clock and VALU activity per ENF_DEBUG_MODE (0 normal, 1 no loads, 2 no loads/stores).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/pmcm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for M in ${MODES:-0 2}; do
  ENF_DEBUG_MODE=$M timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/m$M -o run -- python bench.py --no-cpu --steps 20 --warmup 3 ${BENCH_ARGS:-} > $OUT/m$M.log 2>&1 || { echo "mode $M failed"; tail -5 $OUT/m$M.log; exit 1; }
  python tools/pmc_dispatch.py $OUT/m$M flow_ | tee $OUT/m$M.txt
done
