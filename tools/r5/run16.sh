#!/bin/bash
# round 5, sixteenth GPU pass: PMC of the reference examples' epoch kernel (instructions and waits per step)
set -o pipefail
mkdir -p gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for ex in 2d 1d; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r5/pmc_ex_$ex -o run -- python3 tools/r5/ex_pmc.py $ex > gpurun_out/r5/pmc_ex_$ex.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/r5/pmc2_ex_$ex -o run -- python3 tools/r5/ex_pmc.py $ex > gpurun_out/r5/pmc2_ex_$ex.log 2>&1 || echo "pass 2 failed for $ex"
done
echo ALLDONE
