#!/bin/bash
# round 5, eleventh / twelfth GPU pass: the fp64 in-range forms of the generic gradient kernel (reference examples' training),
# training / VJP / round-4/5 GPU tests, the examples' legs, phase clocks; the fused config-5 step's parts timed
# separately (diagnostics library: ENF_HJG_FUSE=1 with ENF_HJG_FUSE_DBG 0 / 1 wait only / 2 no wait)
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py tests/test_gpu_johnsonsu.py tests/test_gpu_dense_householder.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_vjp.py tests/test_gpu_round4.py tests/test_gpu_round3.py \
  > gpurun_out/r5/pytest_run19.txt 2>&1 || { tail -40 gpurun_out/r5/pytest_run19.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run19.txt
$T 300 python bench_train.py --example 1d > gpurun_out/r5/example_1d_v11.json 2> gpurun_out/r5/example.err || exit 1
$T 300 python bench_train.py --example 2d > gpurun_out/r5/example_2d_v11.json 2>> gpurun_out/r5/example.err || exit 1
$T 120 python tools/r5/small_ts.py 2d 1d > gpurun_out/r5/small_ts_v9.txt 2>&1 || exit 1

echo ALLDONE
