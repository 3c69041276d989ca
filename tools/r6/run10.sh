#!/bin/bash
# round 6, GPU pass 10: the fused gradient kernel's shape at the 8-rank share now that the all-reduce carries its
# rows (fewer blocks = fewer rows to sum in the update launch): variants 0 (product {2,2,8}), 5 {1,2,16}, 4 {1,2,8},
# 3 {2,2,4}, interleaved twice (diagnostics library, ENF_HJG_VARIANT)
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6/c5_share_variants_v1.jsonl
for i in 1 2; do
  for v in 0 5 4 3; do
    ENF_HJG_VARIANT=$v $T 200 python bench_train.py --diag --steps 100 --emulate-world 8 > gpurun_out/r6/v.json 2> gpurun_out/r6/v.err || { tail -5 gpurun_out/r6/v.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6/v.json').read().strip().splitlines()[-1]); print(json.dumps({'variant': $v, 'ms_per_step': d['ms_per_step']}))" >> $P
  done
done
cat $P
