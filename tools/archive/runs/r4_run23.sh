#!/bin/bash
# round 4, twenty-third GPU pass: the D = 64 program with 16 rows per lane (ENF_HJ_R16=1, diagnostics library)
# against the product's 8 rows x 2 columns, interleaved, config-4 shard size (N = 1.25e7), after a settle run
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r4_hj_r16_ab.jsonl
$T 200 python tools/flow_time.py --D 64 --N 12500000 --steps 200 --tag settle >> $P 2>> gpurun_out/r4_hj_r16_ab.err || exit 1
for pass in 1 2 3; do
  for r in 0 1; do
    ENF_HJ_R16=$r $T 200 python tools/flow_time.py --D 64 --N 12500000 --steps 100 --tag r16_$r >> $P 2>> gpurun_out/r4_hj_r16_ab.err || exit 1
  done
done
echo ALLDONE
