#!/bin/bash
# round 4, twenty-first GPU pass: config 2 (J o H, D = 2, N = 1e6, fp64, the compiled D = 2 kernel) under
# rocprofv3 --kernel-trace --stats after the settle phase (the last 50 dispatches are the timed ones)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_c2prof -o run -- python3 bench.py --pattern HJ --D 2 --N 1000000 --dtype f64 --no-cpu --no-train --no-pmc --steps 50 --warmup 5 > gpurun_out/r4_c2prof.log 2>&1 || exit 1
echo ALLDONE
