#!/bin/bash
# round 5, twentieth GPU pass: the fp64 (J o H)^n program under LLVM's scheduler strategies (the fp32 program ships with
# iterative-ilp): libenf.so with only enf_flow_hj64.hip rebuilt per strategy, swapped in on the box, interleaved
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=euclidiannormalizingflows.jl_amd
cp $L/libenf.so $L/libenf_base.so
P=gpurun_out/r5/hj64_sched_ab.jsonl
for rep in 1 2; do
for v in base iterative-ilp max-ilp; do
  if [ $v = base ]; then cp $L/libenf_base.so $L/libenf.so; else cp $L/libenf_hj64_$v.so $L/libenf.so; fi
  $T 300 python bench.py --no-cpu --no-train --no-pmc --dtype f64 --steps 20 --warmup 3 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"$v fwd\"}\t/" >> $P || exit 1
  $T 300 python bench.py --no-cpu --no-train --no-pmc --dtype f64 --inverse --steps 20 --warmup 3 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"$v inv\"}\t/" >> $P || exit 1
done
done
cp $L/libenf_base.so $L/libenf.so
echo ALLDONE
