#!/bin/bash
# round 5, eleventh GPU pass: the fp64 in-range forms of the generic gradient kernel (reference examples' training),
# training / VJP / round-4/5 GPU tests, the examples' legs, phase clocks; the fused config-5 step's parts timed
# separately (diagnostics library: ENF_HJG_FUSE=1 with ENF_HJG_FUSE_DBG 0 / 1 wait only / 2 no wait)
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_round5.py tests/test_gpu_train.py \
  tests/test_gpu_train_semantics.py tests/test_gpu_vjp.py tests/test_gpu_round4.py tests/test_gpu_round3.py \
  > gpurun_out/r5/pytest_run11.txt 2>&1 || { tail -40 gpurun_out/r5/pytest_run11.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run11.txt
$T 300 python bench_train.py --example 1d > gpurun_out/r5/example_1d_v4.json 2> gpurun_out/r5/example.err || exit 1
$T 300 python bench_train.py --example 2d > gpurun_out/r5/example_2d_v4.json 2>> gpurun_out/r5/example.err || exit 1
$T 120 python tools/r5/small_ts.py 2d 1d > gpurun_out/r5/small_ts_v2.txt 2>&1 || exit 1
P=gpurun_out/r5/c5_fuse_ab_v2.jsonl
for dbg in 0 1 2; do
  ENF_HJG_FUSE=1 ENF_HJG_FUSE_DBG=$dbg $T 120 python bench_train.py --diag --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"fuse1_dbg${dbg}_B1e5\"}\t/" >> $P || exit 1
done
ENF_HJG_FUSE=0 $T 120 python bench_train.py --diag --steps 200 --warmup 20 2>/dev/null | tail -1 | sed "s/^/{\"tag\":\"fuse0_B1e5\"}\t/" >> $P || exit 1
echo ALLDONE
