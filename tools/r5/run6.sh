#!/bin/bash
# round 5, sixth GPU pass: the single-block fused step (examples' training legs), the recompute variants of the fused
# (J o H)^n gradient kernel, and the training GPU tests
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_round4.py tests/test_gpu_vjp.py tests/test_gpu_round3.py \
  > gpurun_out/r5/pytest_run6.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run6.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run6.txt
$T 300 python bench_train.py --example 1d > gpurun_out/r5/example_1d_v2.json 2> gpurun_out/r5/example.err || exit 1
$T 300 python bench_train.py --example 2d > gpurun_out/r5/example_2d_v2.json 2>> gpurun_out/r5/example.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof6_ex2d -o ex -- python3 bench_train.py --example 2d > /dev/null 2>&1 || exit 1
echo EXAMPLES_DONE
P=gpurun_out/r5/c5_variants6.jsonl
for v in 0 1 3 5 7 8 9; do
  ENF_HJG_VARIANT=$v $T 120 python bench_train.py --diag --steps 200 --warmup 20 --emulate-world 8 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"v${v}_share8\"}\t/" >> $P || exit 1
  ENF_HJG_VARIANT=$v $T 120 python bench_train.py --diag --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"v${v}_B1e5\"}\t/" >> $P || exit 1
done
echo ALLDONE
