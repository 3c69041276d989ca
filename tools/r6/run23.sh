#!/bin/bash
# round 6, GPU pass 23: a compiled program's first X tile loaded right after the prologue's parameter loads -- training tests, the examples'
# epoch A/B beside round 5's library, and the phase clocks (diagnostics build)
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round6.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_round5.py tests/test_gpu_round4.py > gpurun_out/r6/pytest_run23.txt 2>&1 || { tail -30 gpurun_out/r6/pytest_run23.txt; exit 1; }
tail -1 gpurun_out/r6/pytest_run23.txt
P=gpurun_out/r6/epoch_xafter_ab_v1.jsonl
for i in 1 2; do
  for ex in 2d 1d; do
    $T 200 python tools/epoch_ab.py --example $ex --lib tools/ab/libenf_r5.so --no-zygote-only --tag r5 >> $P || exit 1
    $T 200 python tools/epoch_ab.py --example $ex --tag r6_xafter >> $P || exit 1
  done
done
cat $P
$T 200 python tools/r5/small_ts.py 2d 1d --epoch > gpurun_out/r6/small_ts_epoch_r6_xafter.txt 2>&1 || exit 1
grep -A4 "example" gpurun_out/r6/small_ts_epoch_r6_xafter.txt
