#!/bin/bash
# Round-end measurement refresh on one GPU: full GPU parity suite, smoke(), default bench line (with
# the CPU baseline leg), rocprofv3 kernel-trace stats of the same bench, the other configs, and the
# HBM-traffic PMC passes. Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 20 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
timeout -k 10 300 bash tools/configs.sh > $OUT/configs.log 2>&1 || { tail $OUT/configs.log; exit 1; }
PASSES="FETCH_SIZE;WRITE_SIZE" timeout -k 10 300 bash tools/pmc.sh || exit 1
echo done
