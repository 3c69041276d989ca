#!/bin/bash
# round 5, first GPU pass: (1) the D = 64 16-rows-per-lane A/B (ENF_HJ_R16, diagnostics library) at the config-4
# shard size; (2) config 5 baselines (B = 1e5 fused step, 8-rank share dp step) under rocprofv3 kernel trace
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5/hj_r16_ab.jsonl
$T 200 python tools/flow_time.py --D 64 --N 12500000 --steps 200 --tag settle >> $P 2>> gpurun_out/r5/run1.err || exit 1
for pass in 1 2 3; do
  for r in 0 1; do
    ENF_HJ_R16=$r $T 200 python tools/flow_time.py --D 64 --N 12500000 --steps 100 --tag r16_$r >> $P 2>> gpurun_out/r5/run1.err || exit 1
  done
done
echo R16DONE
$T 300 python bench_train.py --steps 200 --warmup 20 > gpurun_out/r5/c5_B1e5.json 2>> gpurun_out/r5/run1.err || exit 1
$T 300 python bench_train.py --steps 200 --warmup 20 --emulate-world 8 > gpurun_out/r5/c5_share8.json 2>> gpurun_out/r5/run1.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof_c5_share8 -o c5 -- python3 bench_train.py --steps 200 --warmup 20 --emulate-world 8 --graph 0 > gpurun_out/r5/c5_share8_prof.json 2>> gpurun_out/r5/run1.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof_c5_B1e5 -o c5 -- python3 bench_train.py --steps 200 --warmup 20 --graph 0 > gpurun_out/r5/c5_B1e5_prof.json 2>> gpurun_out/r5/run1.err || exit 1
echo ALLDONE
