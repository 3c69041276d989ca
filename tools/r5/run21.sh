#!/bin/bash
# round 5, GPU pass 21: phase clocks of the examples' one-block steps inside the epoch kernel (diagnostics library)
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 180 python tools/r5/small_ts.py 2d 1d --epoch > gpurun_out/r5/small_ts_epoch_v1.txt 2>&1 || exit 1
echo ALLDONE
