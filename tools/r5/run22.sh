#!/bin/bash
# round 5, GPU pass 22 (rerun as 23): the fused barrier-free update of the one-block step
# the reflection scales / row constants: phase clocks, the examples' training legs, the training GPU tests
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 180 python tools/r5/small_ts.py 2d 1d --epoch > gpurun_out/r5/small_ts_epoch_v6.txt 2>&1 || exit 1
$T 300 python bench_train.py --example 1d > gpurun_out/r5/example_1d_v16.json 2> gpurun_out/r5/example.err || exit 1
$T 300 python bench_train.py --example 2d > gpurun_out/r5/example_2d_v16.json 2>> gpurun_out/r5/example.err || exit 1
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_round4.py tests/test_gpu_vjp.py \
  > gpurun_out/r5/pytest_run29.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run29.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run29.txt
echo ALLDONE
