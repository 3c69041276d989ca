#!/bin/bash
# round 5, ninth GPU pass: the fused config-5 step (the reduction inside the gradient launch, enf_grad_hj.h HJFuse):
# training GPU tests, then A/B of fused vs separate reduction launch (diagnostics library, ENF_HJG_FUSE) at the
# 8-rank share and at B = 1e5, and rocprofv3 kernel stats of the product step
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py > gpurun_out/r5/pytest_run9.txt 2>&1 || { tail -40 gpurun_out/r5/pytest_run9.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run9.txt
P=gpurun_out/r5/c5_fuse_ab_v1.jsonl
for rep in 1 2; do
for fz in 1 0; do
  ENF_HJG_FUSE=$fz $T 120 python bench_train.py --diag --steps 200 --warmup 20 --emulate-world 8 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"fuse${fz}_share8\"}\t/" >> $P || exit 1
  ENF_HJG_FUSE=$fz $T 120 python bench_train.py --diag --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"fuse${fz}_B1e5\"}\t/" >> $P || exit 1
done
done
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof9_b -o b -- python3 bench_train.py --steps 200 --warmup 20 > /dev/null 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof9_s -o s -- python3 bench_train.py --steps 200 --warmup 20 --emulate-world 8 > /dev/null 2>&1 || exit 1

T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 120 python tools/r5/small_ts.py 2d 1d > gpurun_out/r5/small_ts_v1.txt 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof10_ex2d -o ex -- python3 bench_train.py --example 2d > /dev/null 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof10_ex1d -o ex -- python3 bench_train.py --example 1d > /dev/null 2>&1 || exit 1
echo ALLDONE
