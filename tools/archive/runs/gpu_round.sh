#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel-trace stats. Stops at the first crash / timeout
# (exit codes other than 0 = pass and 1 = test failures).
set -u
OUT=gpurun_out
mkdir -p $OUT
cd "${GRAFT_REPO_ROOT:-.}"
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
echo "== pytest -m gpu"
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -30 $OUT/pytest_gpu.txt; ok $rc || { echo "pytest crashed rc=$rc"; exit $rc; }
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; [ $rc -eq 0 ] || { echo "bench failed rc=$rc"; exit $rc; }
echo "== rocprofv3 kernel trace"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 20 ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; tail -3 $OUT/prof.err; [ $rc -eq 0 ] || { echo "rocprof failed rc=$rc"; exit $rc; }
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
