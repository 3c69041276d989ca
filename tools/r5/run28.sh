#!/bin/bash
# round 5, GPU pass 28: the cross-lane primitives (permlane swaps, DPP xor tree) against the shuffle butterfly
set -o pipefail
mkdir -p gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 tools/r5/xt/xt > gpurun_out/r5/xt.txt 2>&1; echo "rc=$?" >> gpurun_out/r5/xt.txt
echo ALLDONE
