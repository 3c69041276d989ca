#!/bin/bash
# round 6, GPU pass 6: the shader clock of the headline kernel streaming (ENF_DEBUG_MODE 0) against compute-only
# (2: synthesized tile, no stores) and stores-only (1) -- is the streaming run's extra time a lower clock?
set -o pipefail
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 0 2 1; do
  ENF_DEBUG_MODE=$m timeout -k 10 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/r6/clk$m -o run -- python3 tools/flow_time.py --D 32 --N 10000000 --pairs 4 \
    --steps 30 --tag clk$m > gpurun_out/r6/clk$m.log 2>&1 || { tail -5 gpurun_out/r6/clk$m.log; exit 1; }
done
python3 tools/r6/clk_summary.py gpurun_out/r6/clk0 gpurun_out/r6/clk2 gpurun_out/r6/clk1
