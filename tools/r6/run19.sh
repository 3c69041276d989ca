#!/bin/bash
# round 6, GPU pass 19: VERDICT r05 item 5's trade -- the config-5 share step with the fused gradient kernel's grid
# capped (diagnostics ENF_HJG_MAXBLOCKS) so that its rows would fit the collective (11 rows of 641 doubles <= 64 KiB)
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6/c5_grid_cap_v1.jsonl
for i in 1 2; do
  for m in 0 11 48; do
    ENF_HJG_MAXBLOCKS=$m $T 200 python bench_train.py --diag --steps 100 --emulate-world 8 --breakdown > gpurun_out/r6/v.json 2> gpurun_out/r6/v.err || { tail -5 gpurun_out/r6/v.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6/v.json').read().strip().splitlines()[-1]); print(json.dumps({'max_blocks': $m, 'ms_per_step': d['ms_per_step'], 'phases': d.get('phases')}))" >> $P
  done
done
cat $P
