#!/bin/bash
# round 6, GPU pass 3: placement of the next record's LDS reads in the folded pair loop (ENF_HJ_VAR 0 / 1, the
# diagnostics library) and the compute-only time (ENF_DEBUG_MODE 2: synthesized tile, no stores), config 3
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6/var_ab_v1.jsonl
for i in 1 2 3; do
  for v in 0 1; do
    ENF_HJ_VAR=$v $T 120 python tools/flow_time.py --D 32 --N 10000000 --pairs 4 --steps 100 --tag var$v >> $P || exit 1
  done
done
ENF_DEBUG_MODE=2 $T 120 python tools/flow_time.py --D 32 --N 10000000 --pairs 4 --steps 100 --tag compute_only >> $P || exit 1
ENF_DEBUG_MODE=1 $T 120 python tools/flow_time.py --D 32 --N 10000000 --pairs 4 --steps 100 --tag synth_tile >> $P || exit 1
cat $P
