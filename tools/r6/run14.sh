#!/bin/bash
# round 6, GPU pass 14: the reference examples' epoch with and without ENF_NEGLL_ZYGOTE, beside round 5's library
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6/epoch_zygote_ab_v1.jsonl
for i in 1 2; do
  for ex in 2d 1d; do
    $T 200 python tools/epoch_ab.py --example $ex --lib tools/ab/libenf_r5.so --no-zygote-only --tag r5 >> $P || exit 1
    $T 200 python tools/epoch_ab.py --example $ex --tag r6 >> $P || exit 1
  done
done
cat $P
