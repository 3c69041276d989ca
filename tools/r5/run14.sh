#!/bin/bash
# round 5, fourteenth GPU pass: config 5 at B = 1e5 with 8-wave blocks of 16-byte fragments (ENF_HJG_VARIANT=2: 256
# partial rows instead of 512 for the reduction) against the product shape, interleaved (diagnostics library)
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5/c5_variant2_ab.jsonl
for rep in 1 2; do
for v in 0 2; do
  ENF_HJG_VARIANT=$v $T 120 python bench_train.py --diag --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"v${v}_B1e5\"}\t/" >> $P || exit 1
  ENF_HJG_VARIANT=$v $T 120 python bench_train.py --diag --steps 200 --warmup 20 --emulate-world 8 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"v${v}_share8\"}\t/" >> $P || exit 1
done
done
echo ALLDONE
