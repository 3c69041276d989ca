#!/bin/bash
# round 6, GPU pass 15: the zygote sum taken by the wave that writes the ScaleShift row constants (prologue) --
# tests and the examples' epoch A/B with and without the flag, beside round 5's library
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round6.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_round5.py > gpurun_out/r6/pytest_run15.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run15.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run15.txt
P=gpurun_out/r6/epoch_zygote_ab_v2.jsonl
for i in 1 2; do
  for ex in 2d 1d; do
    $T 200 python tools/epoch_ab.py --example $ex --lib tools/ab/libenf_r5.so --no-zygote-only --tag r5 >> $P || exit 1
    $T 200 python tools/epoch_ab.py --example $ex --tag r6 >> $P || exit 1
  done
done
cat $P
