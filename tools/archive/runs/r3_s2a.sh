#!/bin/bash
# round-3 session-2 first GPU call: trans/FMA mix probe, then the whole GPU suite, smoke, bench, kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/s2a
timeout -k 5 60 ./tools/microbench21 > gpurun_out/s2a/mb21.txt 2>&1 || exit 1
cat gpurun_out/s2a/mb21.txt
R3TAG=s2a bash tools/gpu_r3.sh
