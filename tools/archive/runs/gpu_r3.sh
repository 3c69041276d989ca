#!/bin/bash
# Round-3 GPU session: the whole GPU suite unserialised (per-test time limit), smoke, bench, and the
# rocprofv3 kernel-trace stats of the bench. Stops at the first crash / time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${R3TAG:-r3}
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
echo "== pytest -m gpu"
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.txt; ok $rc || { echo "pytest crashed rc=$rc"; exit $rc; }
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; tail -3 $OUT/smoke.txt; [ $rc -eq 0 ] || { echo "smoke failed rc=$rc"; exit $rc; }
echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; [ $rc -eq 0 ] || { echo "bench failed rc=$rc"; exit $rc; }
echo "== rocprofv3 kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-train --no-pmc --steps 20 ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; tail -3 $OUT/prof.err; [ $rc -eq 0 ] || { echo "rocprof failed rc=$rc"; exit $rc; }
find $OUT/prof -name '*kernel_stats.csv' -exec head -5 {} \;
