#!/bin/bash
# round 5, eighth GPU pass (after the container rebuild): the whole GPU suite, smoke, the headline bench and the
# examples' training legs on the rebuilt libenf.so
set -o pipefail
mkdir -p gpurun_out/r5
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/r5/pytest_run8.txt 2>&1 || { tail -30 gpurun_out/r5/pytest_run8.txt; exit 1; }
tail -2 gpurun_out/r5/pytest_run8.txt
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/smoke_run8.txt 2>&1 || exit 1
$T 300 python bench.py > gpurun_out/r5/bench_v2.json 2> gpurun_out/r5/bench_v2.err || exit 1
$T 300 python bench_train.py --example 1d > gpurun_out/r5/example_1d_v3.json 2> gpurun_out/r5/example.err || exit 1
$T 300 python bench_train.py --example 2d > gpurun_out/r5/example_2d_v3.json 2>> gpurun_out/r5/example.err || exit 1
echo ALLDONE
