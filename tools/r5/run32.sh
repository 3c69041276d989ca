#!/bin/bash
# round 5, GPU pass 32: the whole GPU suite, smoke and the default bench line (with the config-5 train object
# and the reference examples' legs) on the round-5 build
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/r5/pytest_run32_full.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run32_full.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run32_full.txt
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/smoke_run32.txt 2>&1 || exit 1
$T 400 python bench.py > gpurun_out/r5/bench_v7.json 2> gpurun_out/r5/bench_v7.err || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof32 -o b -- python3 bench.py --no-cpu --no-train --no-pmc > /dev/null 2>&1 || exit 1
echo ALLDONE
