#!/bin/bash
# round 5, fifteenth GPU pass: the in-launch reduction again (diagnostics library, ENF_HJG_FUSE=1), now with an
# agent-scope acquire and cached row loads in the reducing blocks, against the two launches; interleaved; plus the
# training GPU tests on the product library
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5/c5_fuse_ab_v3.jsonl
for rep in 1 2; do
for fz in 1 0; do
  ENF_HJG_FUSE=$fz $T 120 python bench_train.py --diag --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"fuse${fz}_B1e5\"}\t/" >> $P || exit 1
  ENF_HJG_FUSE=$fz $T 120 python bench_train.py --diag --steps 200 --warmup 20 --emulate-world 8 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"fuse${fz}_share8\"}\t/" >> $P || exit 1
done
done
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py > gpurun_out/r5/pytest_run18.txt 2>&1 || { tail -40 gpurun_out/r5/pytest_run18.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run18.txt
echo ALLDONE
