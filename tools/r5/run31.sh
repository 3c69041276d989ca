#!/bin/bash
# round 5, GPU pass 31: config 5 with the gradient epilogue's cross-lane sums on permlane swaps / DPP (new) against the
# ds_bpermute shuffles (old), interleaved, at the 8-rank share and at B = 1e5; then the config-5 GPU tests
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=euclidiannormalizingflows.jl_amd
cp $L/libenf.so $L/libenf_c5new.so
P=gpurun_out/r5/c5_xlane_ab.jsonl
for rep in 1 2; do
for v in old new; do
  cp $L/libenf_c5$v.so $L/libenf.so
  $T 120 python bench_train.py --steps 300 --warmup 30 --emulate-world 8 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"${v}_share8\"}\t/" >> $P || exit 1
  $T 120 python bench_train.py --steps 300 --warmup 30 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"${v}_B1e5\"}\t/" >> $P || exit 1
done
done
cp $L/libenf_c5new.so $L/libenf.so
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_round4.py tests/test_gpu_round3.py > gpurun_out/r5/pytest_run31.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run31.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run31.txt
echo ALLDONE
