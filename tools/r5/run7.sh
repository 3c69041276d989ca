#!/bin/bash
# round 5, seventh GPU pass: one-block batches on up to 8 waves (examples' training legs), phase clocks of the
# one-block step (diagnostics library), the training GPU tests
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_round4.py tests/test_gpu_vjp.py tests/test_gpu_round3.py \
  > gpurun_out/r5/pytest_run7.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run7.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run7.txt
$T 300 python bench_train.py --example 1d > gpurun_out/r5/example_1d_v3.json 2> gpurun_out/r5/example.err || exit 1
$T 300 python bench_train.py --example 2d > gpurun_out/r5/example_2d_v3.json 2>> gpurun_out/r5/example.err || exit 1
$T 120 python tools/r5/small_ts.py 2d 1d > gpurun_out/r5/small_ts.txt 2>&1 || exit 1
echo ALLDONE
