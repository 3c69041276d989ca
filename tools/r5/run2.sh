#!/bin/bash
# round 5, second GPU pass: the one-launch reduction + the two-rows-per-lane fused gradient kernel:
# training GPU tests, config-5 step timings (product), the kernel-shape variants (diagnostics library), rocprof
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_round4.py tests/test_gpu_vjp.py tests/test_gpu_round3.py \
  > gpurun_out/r5/pytest_run2.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run2.txt; exit 1; }
tail -3 gpurun_out/r5/pytest_run2.txt
P=gpurun_out/r5/c5_variants.jsonl
for pass in 1 2; do
  $T 120 python bench_train.py --steps 200 --warmup 20 --emulate-world 8 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"prod_share8\"}\t/" >> $P || exit 1
  $T 120 python bench_train.py --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"prod_B1e5\"}\t/" >> $P || exit 1
  for v in 0 1 2 3 4 5; do
    ENF_HJG_VARIANT=$v $T 120 python bench_train.py --diag --steps 200 --warmup 20 --emulate-world 8 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"v${v}_share8\"}\t/" >> $P || exit 1
    ENF_HJG_VARIANT=$v $T 120 python bench_train.py --diag --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"v${v}_B1e5\"}\t/" >> $P || exit 1
  done
done
echo VARIANTS_DONE
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof2_share8 -o c5 -- python3 bench_train.py --steps 200 --warmup 20 --emulate-world 8 --graph 0 > gpurun_out/r5/c5_share8_prof2.json 2>/dev/null || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof2_B1e5 -o c5 -- python3 bench_train.py --steps 200 --warmup 20 --graph 0 > gpurun_out/r5/c5_B1e5_prof2.json 2>/dev/null || exit 1
echo ALLDONE
