#!/bin/bash
# round 5, tenth GPU pass: where the reference examples' one-block step spends its time (phase clocks, diagnostics
# library) and the examples' kernel trace
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 120 python tools/r5/small_ts.py 2d 1d > gpurun_out/r5/small_ts_v1.txt 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof10_ex2d -o ex -- python3 bench_train.py --example 2d > /dev/null 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof10_ex1d -o ex -- python3 bench_train.py --example 1d > /dev/null 2>&1 || exit 1
echo ALLDONE
