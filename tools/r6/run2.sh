#!/bin/bash
# round 6, GPU pass 2: where the folded program's NaN / Inf pattern differs from the oracle's (run 1's failure)
set -o pipefail
mkdir -p gpurun_out/r6
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 120 python tools/r6/dbg_redo.py product 32 > gpurun_out/r6/dbg_redo_r6.txt 2>&1 || exit 1
$T 120 python tools/r6/dbg_redo.py tools/ab/libenf_r5.so 32 > gpurun_out/r6/dbg_redo_r5.txt 2>&1 || exit 1
cat gpurun_out/r6/dbg_redo_r6.txt gpurun_out/r6/dbg_redo_r5.txt
